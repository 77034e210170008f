#!/bin/bash
# int8 LDS layout A/B (development tool): libgsdr.so with fm_am.hip and fir_int8.hip rebuilt with other pad
# periods into build/i8exp/lib<name>.so:  tools/i8_layout_variants.sh <name> <fir P> <chain P>
# (e.g. pad64 64 64 = round 3's layout). Time with tools/ab_ref.py build/i8exp/lib<name>.so
set -e
cd "$(dirname "$0")/.."
NAME=${1:-pad64}; FP=${2:-64}; CP=${3:-64}
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -Iinclude -Igsdr_amd/csrc -munsafe-fp-atomics"
mkdir -p build/i8exp/$NAME
others=$(ls build/*.o | grep -vE '/(fm_am|fir_int8)\.o$')
for f in fm_am fir_int8; do
  /opt/rocm/bin/hipcc $HIPFLAGS -DGSDR_TUNING_PROBES -DGSDR_I8_FIR_PADP=$FP -DGSDR_I8_CHAIN_PADP=$CP -c gsdr_amd/csrc/$f.hip -o build/i8exp/$NAME/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $others build/i8exp/$NAME/fm_am.o build/i8exp/$NAME/fir_int8.o -o build/i8exp/lib$NAME.so
echo built build/i8exp/lib$NAME.so

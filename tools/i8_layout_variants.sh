#!/bin/bash
# int8 LDS layout A/B (development tool): libgsdr.so with fm_am.hip and fir_int8.hip rebuilt with the round-3
# pad period (64 samples) into build/i8exp/libpad64.so. Time with tools/ab_ref.py build/i8exp/libpad64.so
set -e
cd "$(dirname "$0")/.."
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -Iinclude -Igsdr_amd/csrc -munsafe-fp-atomics"
mkdir -p build/i8exp
others=$(ls build/*.o | grep -vE '/(fm_am|fir_int8)\.o$')
for f in fm_am fir_int8; do
  /opt/rocm/bin/hipcc $HIPFLAGS -DGSDR_TUNING_PROBES -DGSDR_I8_FIR_PADP=64 -DGSDR_I8_CHAIN_PADP=64 -c gsdr_amd/csrc/$f.hip -o build/i8exp/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $others build/i8exp/fm_am.o build/i8exp/fir_int8.o -o build/i8exp/libpad64.so
echo built

#!/bin/bash
# Build ablation variants of the IIR (development tool): libgsdr.so with iir.hip recompiled under
# the given -D flags, one library per "name:flags" argument, into build/iirexp/lib<name>.so.
#   tools/iir_variants.sh t1:"-DIIR_PROBE_TAILS=1" f2:"-DIIR_PROBE_FINAL=2"
set -e
cd "$(dirname "$0")/.."
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -Iinclude -Igsdr_amd/csrc -munsafe-fp-atomics"
mkdir -p build/iirexp
others=$(ls build/*.o | grep -v '/iir.o$')
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( /opt/rocm/bin/hipcc $HIPFLAGS -DGSDR_TUNING_PROBES $flags -c gsdr_amd/csrc/iir.hip -o build/iirexp/iir_$name.o &&
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib $others build/iirexp/iir_$name.o \
      -o build/iirexp/lib$name.so && echo "built $name" ) &
done
wait

#!/bin/bash
# Build the product library of an earlier commit (default 50fdf7b, the round-3 tree) into build/ref_<commit>/
# (development tool) so tools/ab_ref.py can time it beside the working tree's library in one process.
set -e
cd "$(dirname "$0")/.."
C=${1:-50fdf7b}
D=build/ref_$C
rm -rf "$D"; mkdir -p "$D/src"
git archive "$C" gsdr_amd/csrc include | tar -x -C "$D/src"
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -I$D/src/include -I$D/src/gsdr_amd/csrc -munsafe-fp-atomics"
objs=""
for f in "$D"/src/gsdr_amd/csrc/*.hip; do
  o="$D/$(basename "$f" .hip).o"; objs="$objs $o"
  /opt/rocm/bin/hipcc $HIPFLAGS -c "$f" -o "$o" &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib $objs -o "$D/libgsdr.so"
echo "built $D/libgsdr.so"

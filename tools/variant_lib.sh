#!/bin/bash
# Build the working tree's library with one translation unit compiled under extra flags (development tool):
#   tools/variant_lib.sh <name> <file.hip> <flags...>   ->  build/var_<name>/libgsdr.so
# The other objects are the product build's (make first). For side-by-side timing with tools/ab_ref.py.
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
D=build/var_$name
mkdir -p "$D"
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -Iinclude -Igsdr_amd/csrc -munsafe-fp-atomics"
b=$(basename "$src" .hip)
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c "$src" -o "$D/$b.o"
objs=$(ls build/*.o | grep -v "/$b.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib $objs "$D/$b.o" -o "$D/libgsdr.so"
echo "built $D/libgsdr.so"

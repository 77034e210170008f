#!/bin/bash
# Build A/B variants of the config-5 kernels (development tool): libgsdr.so with qpsk256.hip from round 3
# (git 50fdf7b, its own awgn.hpp / table) and with the round-4 sources under -DGSDR_AWGN_PAIRS, into
# build/awgnexp/. Time them with: python tools/awgn_time.py build/awgnexp/libr03.so build/awgnexp/libpairs.so
set -e
cd "$(dirname "$0")/.."
HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -fvisibility=hidden -fvisibility-inlines-hidden -Wall -Wno-unused-function -Iinclude -munsafe-fp-atomics"
mkdir -p build/awgnexp/r03
others=$(ls build/*.o | grep -v '/qpsk256.o$')
for f in qpsk256.hip awgn.hpp awgn_table.inc launch.hpp; do git show 50fdf7b:gsdr_amd/csrc/$f > build/awgnexp/r03/$f; done
/opt/rocm/bin/hipcc $HIPFLAGS -Ibuild/awgnexp/r03 -c build/awgnexp/r03/qpsk256.hip -o build/awgnexp/q_r03.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $others build/awgnexp/q_r03.o -o build/awgnexp/libr03.so
/opt/rocm/bin/hipcc $HIPFLAGS -Igsdr_amd/csrc -DGSDR_TUNING_PROBES -DGSDR_AWGN_PAIRS -c gsdr_amd/csrc/qpsk256.hip -o build/awgnexp/q_pairs.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $others build/awgnexp/q_pairs.o -o build/awgnexp/libpairs.so
echo built

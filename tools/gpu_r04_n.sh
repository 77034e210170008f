#!/bin/bash
# Round-4 session N (development tool): final-tree kernel timings and PMC (tools/r04_kernels.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/r04_kernels.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_kernels_final.txt || exit 1
rm -rf gpurun_out/pmc_r04n
bash tools/pmc_cmd.sh pmc_r04n python3 tools/r04_kernels.py > gpurun_out/pmc_r04n.txt 2>&1; rc=$?
tail -5 gpurun_out/pmc_r04n.txt; exit $rc

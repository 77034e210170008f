#!/bin/bash
# Round-4 session B (development tool): GPU suite, float stream timing, PMC of config 5's kernels, the int8
# FM chain and the float FM chain (tools/r04_kernels.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/float_stream_time.py 2>&1 | tee gpurun_out/r04_float_stream_time_b.txt || exit 1
timeout -k 10 120 python -u tools/r04_kernels.py || exit 1
rm -rf gpurun_out/pmc_r04k
bash tools/pmc_cmd.sh pmc_r04k python3 tools/r04_kernels.py > gpurun_out/pmc_r04k.txt 2>&1
tail -40 gpurun_out/pmc_r04k.txt

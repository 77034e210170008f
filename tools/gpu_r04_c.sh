#!/bin/bash
# Round-4 session C (development tool): GPU suite, kernel timings and PMC (tools/r04_kernels.py), kernel trace
# of the float stream timing.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u tools/r04_kernels.py || exit 1
rm -rf gpurun_out/pmc_r04c
bash tools/pmc_cmd.sh pmc_r04c python3 tools/r04_kernels.py > gpurun_out/pmc_r04c.txt 2>&1
grep -E "^[a-z]|LDS_BANK|LDS_IDX|INSTS_VALU|hbm" gpurun_out/pmc_r04c/summary.txt
rm -rf gpurun_out/trace_stream
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_stream -- python3 tools/float_stream_time.py > gpurun_out/trace_stream.log 2>&1
tail -1 gpurun_out/trace_stream.log

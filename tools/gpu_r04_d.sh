#!/bin/bash
# Round-4 session D (development tool): GPU suite, kernel timings, float stream timing and its kernel trace.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
REPS=20 timeout -k 10 180 python -u tools/r04_kernels.py || exit 1
rm -rf gpurun_out/trace_stream
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_stream -- python3 tools/float_stream_time.py > gpurun_out/trace_stream.log 2>&1
grep "us per channel" gpurun_out/trace_stream.log
rm -rf gpurun_out/trace_iir
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_iir -- python3 tools/r04_kernels.py > gpurun_out/trace_iir.log 2>&1
tail -3 gpurun_out/trace_iir.log

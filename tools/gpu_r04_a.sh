#!/bin/bash
# Round-4 session A (development tool): the full GPU suite, then the float stream timing.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/float_stream_time.py 2>&1 | tee gpurun_out/r04_float_stream_time.txt

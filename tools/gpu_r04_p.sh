#!/bin/bash
# Round-4 session P (development tool): int8 / stream / QPSK tests on the final chain layout.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_stream.py tests/test_gpu_multi.py tests/test_gpu_nonfinite.py -m gpu -q -x \
  -p no:cacheprovider --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_p.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_p.log; exit $rc

#!/bin/bash
# Round-4 session F (development tool): GPU suite, then the working tree against the round-3 library side by
# side (tools/ab_ref.py) and the config-5 table-layout A/B (tools/awgn_time.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_ref.py build/ref_50fdf7b/libgsdr.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_ref.txt || exit 1
timeout -k 10 200 python -u tools/awgn_time.py build/awgnexp/libpairs.so build/awgnexp/libr03.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_awgn_ab.txt

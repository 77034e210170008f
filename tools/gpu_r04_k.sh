#!/bin/bash
# Round-4 session K (development tool): AWGN NaN-sentinel tail test; QPSK tests and A/B against round 3.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_qpsk.py -m gpu -q -x -p no:cacheprovider --timeout 200 \
  --timeout-method thread -rf > gpurun_out/pytest_k.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_k.log; [ $rc = 0 ] || exit $rc
ROUNDS=10 CASES=gsdrxQpsk256ModulateAwgn,gsdrQpsk256Demodulate,gsdrxFmDemodInt8 \
  timeout -k 10 400 python -u tools/ab_ref.py build/ref_50fdf7b/libgsdr.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_k.txt

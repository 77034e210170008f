#!/bin/bash
# Round-4 session I (development tool): int8 short-call tile shapes, chain pad-period and AWGN A/B, int8/QPSK tests.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_qpsk.py -m gpu -q -x -p no:cacheprovider \
  --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_i.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_i.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/short_call_i8.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_short_i8.txt || exit 1
ROUNDS=6 CASES=gsdrxFirFCInt8,gsdrxFmDemodInt8,gsdrxAmDemodInt8,gsdrxQpsk256ModulateAwgn,gsdrQpsk256Demodulate \
  timeout -k 10 400 python -u tools/ab_ref.py build/i8exp/libc32.so build/i8exp/libc64.so build/ref_50fdf7b/libgsdr.so 2>&1 \
  | grep -v amdgpu.ids | tee gpurun_out/r04_ab_i.txt

#!/bin/bash
# Round-4 session J (development tool): int8 tap-row gather and first-tile early loads; int8/QPSK/stream tests,
# short-call timing and A/B against the round-3 library.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_qpsk.py tests/test_gpu_stream.py -m gpu -q -x \
  -p no:cacheprovider --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_j.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_j.log; [ $rc = 0 ] || exit $rc
VARIANTS=41,43,45 timeout -k 10 200 python -u tools/short_call_i8.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_short_i8_j.txt || exit 1
ROUNDS=8 CASES=gsdrxFirFCInt8,gsdrxFmDemodInt8,gsdrxAmDemodInt8,gsdrxQpsk256ModulateAwgn,gsdrQpsk256Demodulate \
  timeout -k 10 400 python -u tools/ab_ref.py build/ref_50fdf7b/libgsdr.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_j.txt

#!/bin/bash
# Round-4 session G (development tool): int8 layout and AWGN A/B against the round-3 library, then the suite.
mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=6 CASES=gsdrxFirFCInt8,gsdrxFmDemodInt8,gsdrxAmDemodInt8,gsdrxQpsk256ModulateAwgn,gsdrQpsk256Demodulate \
  timeout -k 10 400 python -u tools/ab_ref.py build/i8exp/libpad64.so build/ref_50fdf7b/libgsdr.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_g.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
bash tools/gpu_r04_h.sh

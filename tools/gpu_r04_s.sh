#!/bin/bash
# Round-4 session S (development tool): int8 FM discriminator with the rotation folded into the products;
# int8 tests, then side by side with the previous build.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_stream.py tests/test_gpu_multi.py tests/test_gpu_nonfinite.py -m gpu -q -x \
  -p no:cacheprovider --timeout 200 --timeout-method thread -rf > gpurun_out/pytest_s.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_s.log; [ $rc = 0 ] || exit $rc
ROUNDS=10 CASES=gsdrxFmDemodInt8,gsdrxAmDemodInt8 timeout -k 10 300 python -u tools/ab_ref.py build/rotexp/libbefore.so 2>&1 \
  | grep -v amdgpu.ids | tee gpurun_out/r04_ab_s.txt

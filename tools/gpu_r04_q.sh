#!/bin/bash
# Round-4 session Q (development tool): IIR tile rows at an odd float stride; IIR tests, A/B and PMC.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_iir.py -m gpu -q -x -p no:cacheprovider --timeout 200 \
  --timeout-method thread -rf > gpurun_out/pytest_q.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_q.log; [ $rc = 0 ] || exit $rc
ROUNDS=10 CASES=gsdrIirFF,gsdrIirCC timeout -k 10 300 python -u tools/ab_ref.py build/iirexp/libbefore.so 2>&1 \
  | grep -v amdgpu.ids | tee gpurun_out/r04_ab_q.txt

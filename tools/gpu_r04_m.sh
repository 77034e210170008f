#!/bin/bash
# Round-4 session M (development tool): config-5 kernels before / after the power-capped FIR; QPSK tests.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_qpsk.py -m gpu -q -x -p no:cacheprovider --timeout 200 \
  --timeout-method thread -rf > gpurun_out/pytest_m.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_m.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/thermal_order.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_thermal_order.txt

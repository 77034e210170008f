#!/bin/bash
# Round-4 closing check (development tool): the whole GPU suite and smoke() on the final tree.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf \
  > gpurun_out/pytest_gpu_final.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_final.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1

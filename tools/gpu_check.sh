#!/bin/bash
# One GPU session: tests, smoke, bench. Stops at the first crash-like exit status
# (abort 134, segfault 139, timeout 124/137); ordinary test failures (exit 1) do not stop the bench.
mkdir -p gpurun_out
ok() { case "$1" in 0|1|2|5) return 0;; *) echo "stopping: exit status $1"; return 1;; esac; }
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/bench.log
exit $rc

#!/bin/bash
# Development session: the named GPU test files first (stop on failure), then the whole GPU suite,
# smoke and a bench line. Stops at the first crash-like exit status.
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) echo "stopping: exit status $1"; return 1;; esac; }
timeout -k 10 600 python -u -m pytest ${NEW_TESTS} -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "new tests exit $rc"; tail -15 gpurun_out/pytest_new.log; [ $rc = 0 ] || exit $rc
[ -n "${ONLY_NEW}" ] && exit 0
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/bench.log
exit $rc

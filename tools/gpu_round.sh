#!/bin/bash
# Round evidence session: GPU tests, smoke, bench, rocprofv3 stats of the same bench command,
# separate PMC passes for HBM traffic. Stops at the first crash-like exit status.
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { case "$1" in 0|1) return 0;; *) echo "stopping: exit status $1"; return 1;; esac; }
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 gpurun_out/smoke.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -1 gpurun_out/bench.log; [ $rc = 0 ] || exit $rc
rm -rf gpurun_out/prof_bench gpurun_out/pmc_bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -- python bench.py > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof bench exit $rc"; [ $rc = 0 ] || exit $rc
grep kernel_us_mean gpurun_out/prof_bench.log | tail -1 > gpurun_out/bench_profiled.json  # the profiled run's own line
bash tools/pmc.sh pmc_bench python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > gpurun_out/pmc_bench.log 2>&1
rc=$?; echo "pmc exit $rc"; tail -25 gpurun_out/pmc_bench.log
exit $rc

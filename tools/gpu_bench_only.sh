mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench2.log 2>&1; rc=$?; tail -1 gpurun_out/bench2.log | cut -c1-300; exit $rc

#!/bin/bash
# usage: tools/gpu_run.sh <tag> <step>...   (run on the GPU box through gpurun)
# Steps, in order, each under its own time limit; output under gpurun_out/<tag>_*. Stops after any crash-like
# exit status (only 0 and pytest's 1 = "tests failed" continue):
#   tests:<pytest args>   python -m pytest -m gpu <args>
#   bench[:<args>]        python bench.py <args>
#   smoke                 __graft_entry__.smoke()
#   prof[:<args>]         rocprofv3 --kernel-trace --stats of python bench.py <args>
#   pmc[:<args>]          tools/pmc.sh of python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline <args>
#   py:<script> [args]    python <script> <args>
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
cont() { case "$1" in 0|1) return 0;; *) echo "stopping: exit status $1"; return 1;; esac; }
i=0
for step in "$@"; do
  i=$((i+1))
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  log=gpurun_out/${tag}_${i}_${kind}.log
  case $kind in
    tests) timeout -k 10 1100 python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf $arg > $log 2>&1 ;;
    bench) timeout -k 10 600 python bench.py $arg > $log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 ;;
    prof) rm -rf gpurun_out/${tag}_prof; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -- python bench.py $arg > $log 2>&1 ;;
    pmc) bash tools/pmc.sh ${tag}_pmc python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline $arg > $log 2>&1 ;;
    py) timeout -k 10 600 python -u $arg > $log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $i $kind exit $rc"; tail -3 $log
  cont $rc || exit $rc
done

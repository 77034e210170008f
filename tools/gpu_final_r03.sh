#!/bin/bash
# Round-3 closing session: IIR A/B against the given build, the round evidence (tools/gpu_round.sh), and the
# k_fir_rt PMC at D = 50 / 13 (tools/pmc.sh over tools/fir_rt_probe.py). Stops at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/iir_exp.sh "$@" > gpurun_out/iir_exp4.txt 2>&1; rc=$?; cat gpurun_out/iir_exp4.txt; [ $rc = 0 ] || exit $rc
rm -rf gpurun_out/prof_bench gpurun_out/pmc_bench
bash tools/gpu_round.sh || exit $?
for d in 50 13; do
  rm -rf gpurun_out/firrt$d
  bash tools/pmc.sh firrt$d python3 tools/fir_rt_probe.py $d > gpurun_out/firrt$d.txt 2>&1 || exit $?
  grep "gsdrFirFC" gpurun_out/firrt$d/trace.log
  grep -E "k_fir_rt|LDS_BANK|LDS_IDX" gpurun_out/firrt$d.txt
done

#!/bin/bash
# Energy per launch of the headline FIR and its ablations (verdict r01 item 7), then the bench line with
# the staging ceiling. Development session script for gpurun.
mkdir -p gpurun_out
LAUNCHES=${LAUNCHES:-30000} bash tools/power_split.sh ${VARIANTS:-0 13 14 104 107 int8:0} > gpurun_out/power_split.txt 2>&1 || { cat gpurun_out/power_split.txt; exit 1; }
cat gpurun_out/power_split.txt
python tools/energy_table.py gpurun_out/power_split.txt | tee gpurun_out/energy_table.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench.log; exit $rc

#!/bin/bash
# Probe session: variant sweep, then rocprofv3 kernel-trace stats and PMC passes on the probe.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/fir_probe.py --fm > gpurun_out/probe.log 2>&1 || { echo "probe failed $?"; exit 1; }
cat gpurun_out/probe.log
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
P="python tools/fir_probe.py --variants 0,100,101,102 --reps 3 --rounds 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -- $P > gpurun_out/prof_trace.log 2>&1 || { echo "trace failed"; exit 1; }
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc$i -- $P > gpurun_out/pmc$i.log 2>&1 || { echo "pmc pass $i failed ($C)"; tail -5 gpurun_out/pmc$i.log; }
done
echo done

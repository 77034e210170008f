#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, never combined with tracing) over any command.
# usage: tools/pmc_cmd.sh <outdir-under-gpurun_out> <command...>
out=gpurun_out/$1; shift
mkdir -p "$out"; export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$out/pmc$i" -- "$@" > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed ($C)"; tail -3 "$out/pmc$i.log"; }
done
python3 tools/pmc_summary.py "$out" > "$out/summary.txt"
cat "$out/summary.txt"

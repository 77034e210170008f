#!/bin/bash
# usage: tools/pmc.sh <outdir-under-gpurun_out> <command...>
# rocprofv3 kernel-trace/stats pass, then separate PMC passes (never combined with tracing).
out=gpurun_out/$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -- "$@" > "$out/trace.log" 2>&1 || { echo "trace pass failed"; exit 1; }
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$out/pmc$i" -- "$@" > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed ($C)"; tail -3 "$out/pmc$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$out" --json "$out/summary.json" > "$out/summary.txt"
cat "$out/summary.txt"

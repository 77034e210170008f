#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, never combined with tracing) over fir_probe.py
# for the listed gsdrxFirFCVariant values. usage: tools/pmc_variants.sh <outdir> <variants>
out=gpurun_out/$1; v=$2
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" \
         "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$out/pmc$i" -- python3 tools/fir_probe.py --variants $v --reps 5 --rounds 1 > "$out/pmc$i.log" 2>&1 || { echo "pmc pass $i failed ($C)"; tail -3 "$out/pmc$i.log"; }
done
python3 tools/pmc_summary.py "$out" > "$out/summary.txt"
cat "$out/summary.txt"

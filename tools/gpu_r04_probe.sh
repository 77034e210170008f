#!/bin/bash
# Round-4 probe session (development tool, run through gpurun): LDS-read probe of the headline FIR
# (140/141 vs 0/104) and the tile-relative NCO probe of the FM chain (127 vs 120/126), interleaved
# timing, then the power split of the FIR variants.
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/rel_nco_check.py || exit 1
timeout -k 10 300 python -u tools/fir_probe.py --variants 0,140,104,141,107,120,127,126,121 --rounds 5 \
  > gpurun_out/r04_probe_time.txt 2>&1 || { cat gpurun_out/r04_probe_time.txt; exit 1; }
cat gpurun_out/r04_probe_time.txt
LAUNCHES=${LAUNCHES:-15000} bash tools/power_split.sh 0 140 104 141 107 > gpurun_out/power_split.txt 2>&1 || { cat gpurun_out/power_split.txt; exit 1; }
cat gpurun_out/power_split.txt
python tools/energy_table.py gpurun_out/power_split.txt | tee gpurun_out/r04_energy_table.txt

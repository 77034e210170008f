#!/bin/bash
# FM chain (config 3 shape) energy split (development tool): interleaved timing of the FM-mode
# ablations of the probes build (120 full, 121 no NCO mix, 122 no discriminator, 123 neither,
# 124 staging + NCO + discriminator without the FIR, 125 staging only, 126 NCO mix without its
# transcendental pair) beside the FIR (0) and FIR staging only (107), then power / sclk per variant.
mkdir -p gpurun_out
timeout -k 10 300 python tools/fir_probe.py --variants ${FM_VARIANTS:-0,107,120,121,122,123,124,125,126} --reps 50 --rounds 5 \
  > gpurun_out/fm_split_time.txt 2>&1 || { cat gpurun_out/fm_split_time.txt; exit 1; }
cat gpurun_out/fm_split_time.txt
bash tools/power_split.sh ${FM_POWER:-0 120 121 122 123 125 126} | tee gpurun_out/fm_split_power.txt

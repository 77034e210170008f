#!/bin/bash
# Power / clock of the FIR ablations (development tool): compute-only (104), staging-only nt (107),
# full kernel nt (106). Prints steady us/launch and the power / sclk samples taken during each run.
for v in "$@"; do
  rm -f gpurun_out/clock_watch.log
  timeout -k 10 200 bash tools/clock_watch.sh "$v" 8000 || exit 1
  echo "power W:" $(grep -oE "Package Power \(W\): [0-9.]+" gpurun_out/clock_watch.log | awk '{print $NF}' | sort -n | tail -8 | tr '\n' ' ')
  echo "sclk MHz:" $(grep -oE "sclk clock level: [0-9]+: \([0-9]+Mhz\)" gpurun_out/clock_watch.log | grep -oE "[0-9]+Mhz" | tr '\n' ' ')
done

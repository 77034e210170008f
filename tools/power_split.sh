#!/bin/bash
# Power / clock of the headline FIR and its ablations (development tool). Arguments are variants of
# gsdrxFirFCVariant (e.g. 104 = compute only, 107 = staging only, 0 = full kernel) or "int8:V" for
# gsdrxFirFCInt8Variant. For each: steady us/launch, then the package power and sclk samples that
# rocm-smi reported while it ran (sampled ~4x per second); the raw samples stay in
# gpurun_out/clock_watch_<arg>.log for tools/energy_table.py. LAUNCHES (default 8000) per variant.
for arg in "$@"; do
  v=${arg#int8:}
  extra=""
  [ "$v" != "$arg" ] && extra="--int8"
  rm -f gpurun_out/clock_watch.log
  echo "== $arg"
  EXTRA=$extra timeout -k 10 200 bash tools/clock_watch.sh "$v" "${LAUNCHES:-8000}" | grep variant || exit 1
  cp gpurun_out/clock_watch.log "gpurun_out/clock_watch_${arg/:/_}.log"
  echo "  power W (top 8):" $(grep -oE "Package Power \(W\): [0-9.]+" gpurun_out/clock_watch.log | awk '{print $NF}' | sort -n | tail -8 | tr '\n' ' ')
  echo "  sclk MHz:" $(grep -oE "sclk clock level: [0-9]+: \([0-9]+Mhz\)" gpurun_out/clock_watch.log | grep -oE "[0-9]+Mhz" | tr '\n' ' ')
done

#!/bin/bash
# Kernel-trace stats of 20 IIR calls, real and complex (development tool).
mkdir -p gpurun_out; export TMPDIR=/tmp
for k in ${IIR_KINDS:-ff cc}; do
  rm -rf gpurun_out/iirprof_$k
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iirprof_$k -- python3 tools/iir_probe.py $k ${IIR_LOG2N:-24} > gpurun_out/iirprof_$k.log 2>&1 || exit $?
  f=$(find gpurun_out/iirprof_$k -name "*kernel_stats.csv" | head -1)
  echo "== $k"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('%-60s %6s calls  avg %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
done

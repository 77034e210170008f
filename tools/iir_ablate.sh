#!/bin/bash
# Per-kernel kernel-trace means of gsdrIirFF / CC (20 calls, 2^24 samples) for the in-tree build and
# each build/iirexp/lib<name>.so given by name (development tool; tools/iir_variants.sh builds them).
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base "$@"; do
  lib=gsdr_amd/libgsdr.so; [ "$v" = base ] || lib=build/iirexp/lib$v.so
  for k in ${IIR_KINDS:-ff}; do
    d=gpurun_out/iirabl_${v}_$k; rm -rf $d
    GSDR_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python3 tools/iir_probe.py $k ${IIR_LOG2N:-24} > $d.log 2>&1 || { echo "failed $v $k"; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    echo "== $v $k"; python3 -c "
import csv
tot=0
for r in csv.DictReader(open('$f')):
    a=float(r['AverageNs'])/1e3; tot+=a*int(r['Calls'])/20
    print('  %-70s %4s  %8.2f us' % (r['Name'][:70], r['Calls'], a))
print('  per call (sum of kernel means) %.2f us' % tot)"
  done
done

#!/bin/bash
# Kernel-trace of the int8 stream at C chunks a pass (development tool): per-launch duration and the gap
# between launches of the matrix-core kernel.  usage: tools/stream_trace.sh [chunks]
mkdir -p gpurun_out; export TMPDIR=/tmp
c=${1:-32}; d=gpurun_out/s$c; rm -rf $d
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python3 tools/int8_stream_probe.py $c > $d.log 2>&1 || exit $?
f=$(find $d -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, statistics as S, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "i8_mfma" in r["Kernel_Name"]]
st = [int(r["Start_Timestamp"]) for r in rows]; en = [int(r["End_Timestamp"]) for r in rows]
d = [(b - a) / 1e3 for a, b in zip(st, en)]
g = [(st[i + 1] - en[i]) / 1e3 for i in range(len(st) - 1)]
print(len(d), "launches; duration median %.2f us (min %.2f), gap median %.2f us" % (S.median(d[-100:]), min(d), S.median(g[-100:])))
print(rows[-1]["Kernel_Name"][:90], "grid", rows[-1].get("Grid_Size"), "wg", rows[-1].get("Workgroup_Size"))
PY

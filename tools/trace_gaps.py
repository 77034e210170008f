#!/usr/bin/env python3
"""Split the kernel trace of examples/short_call_timer.cpp into per-call kernel duration and launch gap
(development tool):
    rocprofv3 --kernel-trace --output-format csv -d <dir> -- ./build/short_call_timer <calls>
    python tools/trace_gaps.py <dir> <calls>
The timer issues, in order: 300 warm-up gsdrFmDemod calls, <calls> gsdrMagnitude(256), then for 2^16, 2^18, 2^20
samples <calls> direct gsdrFmDemod calls and <calls> gsdrxStreamProcess calls (one launch each). For each segment
it prints the median kernel duration, the median gap from a kernel's end to the next kernel's start, and their
sum (the per-call period the HIP events measure)."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, calls = sys.argv[1], int(sys.argv[2])
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    assert files, f"no kernel_trace.csv under {d}"
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows = [r for r in rows if "gsdr::" in r["Kernel_Name"]]  # (the runtime's own copy / fill blits aside)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs = [("warmup", 300), ("gsdrMagnitude_256", calls)]
    for n in (1 << 16, 1 << 18, 1 << 20):
        segs += [(f"gsdrFmDemod_{n}", calls), (f"gsdrxStreamProcess_fm_{n}", calls)]
    want = sum(c for _, c in segs)
    assert len(rows) == want, f"{len(rows)} dispatches in the trace, expected {want} (one launch a call)"
    out, i = [], 0
    for name, c in segs:
        seg = rows[i:i + c]
        i += c
        if name == "warmup":
            continue
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg]
        gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:])]
        md, mg = statistics.median(dur), statistics.median(gap)
        out.append({"segment": name, "kernel": seg[0]["Kernel_Name"][:90], "kernel_us_median": round(md, 3),
                    "gap_us_median": round(mg, 3), "period_us": round(md + mg, 3),
                    "kernel_us_p10_p90": [round(sorted(dur)[len(dur) // 10], 3), round(sorted(dur)[9 * len(dur) // 10], 3)]})
        print(f"{name:30s} kernel {md:7.3f} us   gap {mg:7.3f} us   period {md + mg:7.3f} us   {seg[0]['Kernel_Name'][:60]}")
    print(json.dumps(out))


if __name__ == "__main__":
    main()

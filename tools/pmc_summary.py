#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace stats + PMC passes) per kernel.

usage: tools/pmc_summary.py <dir-with-rocprofv3-output> [--json out.json] [--filter substr]
Per kernel: dispatches, mean duration (kernel trace), mean of each PMC counter per dispatch, and the
derived HBM bytes per dispatch using the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reads
half the bytes of a wide coalesced stream: x2; WRITE_SIZE exact; both in KiB).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name):
    name = re.sub(r"HIP_vector_type<float, 2u>", "f2", name)
    name = re.sub(r"\(gsdr::FirParams.*", "", name)
    return name.replace("gsdr::", "")[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--filter", default="gsdr")
    a = ap.parse_args()
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.filter not in r["Kernel_Name"]:
                continue
            counters[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.filter not in r["Kernel_Name"]:
                continue
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    out = {}
    for k in sorted(set(counters) | set(durs)):
        d = {c: sum(v) / len(v) for c, v in counters[k].items()}
        if durs[k]:
            d["dispatches"] = len(durs[k])
            d["duration_us_mean"] = sum(durs[k]) / len(durs[k])
        if "FETCH_SIZE" in d or "WRITE_SIZE" in d:
            d["hbm_bytes_corrected"] = (2 * d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) * 1024
        out[k] = d
        print(k)
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v:,.1f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

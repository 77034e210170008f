#!/usr/bin/env python3
"""Copy the round's rocprofv3 evidence into profiles/ (tracked):
  profiles/<tag>_bench_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `python bench.py`
  profiles/<tag>_pmc_summary.json         per-kernel PMC means (tools/pmc_summary.py)
  profiles/pmc_fir_fc_d4.json             HBM bytes per launch of the headline kernel, read by bench.py
usage: tools/make_profile_summary.py <tag> [--kernel substr]
"""
import argparse
import glob
import json
import os
import shutil
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--kernel", default="void k_fir_poly<float, f2, 4, 4, 16, 256, true, 0, 0, true, false, 0, false, false>")
ap.add_argument("--stats-dir", default="gpurun_out/prof_bench")
ap.add_argument("--pmc-dir", default="gpurun_out/pmc_bench")
ap.add_argument("--steps", type=int, default=100, help="timed steps of the profiled bench run")
a = ap.parse_args()
prof = os.path.join(ROOT, "profiles")
os.makedirs(prof, exist_ok=True)
stats = sorted(glob.glob(os.path.join(ROOT, a.stats_dir, "**", "*kernel_stats.csv"), recursive=True),
               key=os.path.getmtime)
timed_mean = None
if stats:
    shutil.copy(stats[-1], os.path.join(prof, f"{a.tag}_bench_kernel_stats.csv"))
    trace = stats[-1].replace("kernel_stats.csv", "kernel_trace.csv")
    import csv
    fir_name = "void gsdr::" + a.kernel[len("void "):].replace("f2", "HIP_vector_type<float, 2u>")
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in csv.DictReader(open(trace))
         if r["Kernel_Name"].startswith(fir_name)]
    if d:
        # the timed steps are dispatches [W + settle, W + settle + K) of the headline kernel: the profiled run's
        # own line says how many warm-up and clock-settle launches preceded them
        lo, what = len(d) - a.steps, f"the last {a.steps}"
        pl = os.path.join(ROOT, "gpurun_out", "bench_profiled.json")
        if os.path.exists(pl):
            line = json.loads(open(pl).read().strip().splitlines()[-1])
            lo = int(line.get("warmup", 0)) + int(line.get("clock_settle_launches", 0))
            what = f"dispatches {lo}..{lo + a.steps - 1} (after {line.get('warmup')} warm-up and {line.get('clock_settle_launches')} clock-settle launches)"
        w = d[lo:lo + a.steps]
        timed_mean = sum(w) / len(w)
        with open(os.path.join(prof, f"{a.tag}_bench_fir_dispatches.txt"), "w") as f:
            f.write(f"# {fir_name}: per-dispatch duration (us) from rocprofv3 --kernel-trace of `python bench.py`\n")
            f.write(f"# dispatches {len(d)}; the timed steps = {what}: mean {timed_mean:.2f} us\n")
            f.write("\n".join(f"{x:.2f}" for x in d) + "\n")
prof_line = os.path.join(ROOT, "gpurun_out", "bench_profiled.json")
if os.path.exists(prof_line):  # the profiled run's own bench line (gpu_round.sh), to set beside the trace
    shutil.copy(prof_line, os.path.join(prof, f"{a.tag}_bench_line_profiled.json"))
summ = json.load(open(os.path.join(ROOT, a.pmc_dir, "summary.json")))
shutil.copy(os.path.join(ROOT, a.pmc_dir, "summary.json"), os.path.join(prof, f"{a.tag}_pmc_summary.json"))
k = summ[a.kernel]
out = {
    "kernel": a.kernel,
    "hbm_bytes_per_launch": round(k["hbm_bytes_corrected"]),
    "fetch_size_kib": k["FETCH_SIZE"],
    "write_size_kib": k["WRITE_SIZE"],
    "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE reports half the bytes "
                  "of a wide coalesced stream, WRITE_SIZE is exact (MI355X_MICROARCH.md, HBM section)",
    "pmc_duration_us_mean": k.get("duration_us_mean"),
    "rocprof_timed_steps_us_mean": timed_mean,
    "command": "tools/pmc.sh pmc_bench python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline "
               "(one rocprofv3 --pmc pass per counter group)",
    "round": a.tag,
    "generated": time.strftime("%Y-%m-%d %H:%M:%S"),
}
json.dump(out, open(os.path.join(prof, "pmc_fir_fc_d4.json"), "w"), indent=1)
print(json.dumps(out, indent=1))

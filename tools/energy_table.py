#!/usr/bin/env python3
"""Energy per launch from a tools/power_split.sh session (development tool).

    python tools/energy_table.py gpurun_out/power_split.txt

For each variant: the steady per-launch time (sustained_probe's last window), the median package power
over the samples taken while the kernel ran (samples above 60 % of that log's peak: rocm-smi keeps
sampling before the launches start and after they end), and energy per launch = power x time, total and
above the idle floor (the log's lowest sample)."""
import re
import statistics
import sys


def main(path):
    text = open(path).read()
    rows = []
    for block in text.split("== ")[1:]:
        arg = block.split()[0]
        m = re.search(r"steady ([0-9.]+) us", block)
        if not m:
            continue
        us = float(m.group(1))
        try:
            pw = [float(x) for x in re.findall(r"Package Power \(W\): ([0-9.]+)",
                                               open(f"gpurun_out/clock_watch_{arg.replace(':', '_')}.log").read())]
        except OSError:
            continue
        if not pw:
            continue
        hi = [p for p in pw if p >= 0.6 * max(pw)]
        rows.append((arg, us, statistics.median(hi), min(pw), len(hi)))
    print(f"{'variant':>8} {'us':>8} {'W (run)':>8} {'W idle':>7} {'mJ total':>9} {'mJ dyn':>7} {'samples':>7}")
    for key, us, p, p0, n in rows:
        print(f"{key:>8} {us:8.1f} {p:8.0f} {p0:7.0f} {p * us * 1e-3:9.1f} {(p - p0) * us * 1e-3:7.1f} {n:7d}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/power_split.txt")

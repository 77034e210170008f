#!/usr/bin/env python3
"""Print the headline and every secondary timing of a bench.py JSON line (development tool).

    python tools/bench_summary.py gpurun_out/bench.log
"""
import json
import sys


def main(path):
    line = [ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    r = d["roofline"]
    print(f"headline {r['kernel_us_mean']} us frac {r['frac']} value {d['value']} {d['unit']}"
          f" staging {r.get('staging_ceiling', {}).get('us')} copy {r.get('measured_copy_gbps')}")
    for k, v in d.get("secondary", {}).items():
        flat = {kk: vv for kk, vv in v.items() if isinstance(vv, (int, float)) and ("us" in kk or "frac" in kk)}
        print(f"  {k}: {flat}")
        for kk, vv in v.items():
            if isinstance(vv, dict) and ("chunks" in kk or "per_call" in kk):
                print(f"      {kk}: us/call {vv.get('us_per_call')} pass {vv.get('us_per_pass')} "
                      f"vs_single {vv.get('vs_single_call')} host {vv.get('host_us_per_call')}")
    if "multi_gpu_check" in d:
        print("  multi:", d["multi_gpu_check"])


if __name__ == "__main__":
    main(sys.argv[1])

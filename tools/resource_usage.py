#!/usr/bin/env python3
"""Compile one .hip file with -Rpass-analysis=kernel-resource-usage and print a per-kernel table
(VGPRs, SGPRs, scratch, occupancy). Development aid, not part of the library."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", "-Iinclude",
       "-Igsdr_amd/csrc", "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (?:\S+: )?\s*(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split()[0]] = v
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.splitlines()
for r, n in zip(rows, names):
    n = n.replace("HIP_vector_type<float, 2u>", "f2").replace("gsdr::", "").replace("(FirParams)", "")
    print(f"{r.get('VGPRs','?'):>4} v {r.get('AGPRs','0'):>3} a {r.get('TotalSGPRs','?'):>3} s scr={r.get('ScratchSize','?'):>4} occ={r.get('Occupancy','?')}  {n}")

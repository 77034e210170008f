#!/bin/bash
# Round-4 session R (development tool): where the int8 FM chain's time goes (probe builds: 1 = no exchange and
# no discriminator, 2 = exchange and products, no angle), side by side with the library order rotated.
mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=10 CASES=gsdrxFmDemodInt8,gsdrxAmDemodInt8,gsdrxFirFCInt8 timeout -k 10 300 python -u tools/ab_ref.py \
  build/fmprobe/libp1.so build/fmprobe/libp2.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_r.txt

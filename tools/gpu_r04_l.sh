#!/bin/bash
# Round-4 session L (development tool): int8 multi-channel per-channel matrix-core launches vs the grouped kernel.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/multi_int8_time.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_multi_int8.txt

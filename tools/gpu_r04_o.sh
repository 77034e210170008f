#!/bin/bash
# Round-4 session O (development tool): chain pad period and AWGN table layout, side by side with the library
# order rotated every round.
mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=10 CASES=gsdrxFmDemodInt8,gsdrxAmDemodInt8,gsdrxQpsk256ModulateAwgn,gsdrQpsk256Demodulate \
  timeout -k 10 500 python -u tools/ab_ref.py build/i8exp/libc16.so build/i8exp/libc64.so build/awgnexp/libpairs.so \
  build/awgnexp/libr03.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04_ab_o.txt

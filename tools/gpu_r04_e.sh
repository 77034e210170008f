#!/bin/bash
# Round-4 session E (development tool): short-call tile shapes under a kernel trace, IIR timing.
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/trace_shapes
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_shapes -- python3 tools/short_call_shapes.py > gpurun_out/trace_shapes.log 2>&1 || exit 1
grep "N =" gpurun_out/trace_shapes.log
REPS=20 timeout -k 10 180 python -u tools/r04_kernels.py || exit 1

#!/bin/bash
# Round-4 session H (development tool): int8 short-call tile sizes under a kernel trace.
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/trace_i8short
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_i8short -- python3 tools/short_call_i8.py > gpurun_out/trace_i8short.log 2>&1 || exit 1
grep "N =" gpurun_out/trace_i8short.log

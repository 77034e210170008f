#!/bin/bash
# examples/short_call_timer (C++ back-to-back calls) of this tree against an earlier build's timer
# (build/short_call_timer_ref, linked to build/ref_<commit>/libgsdr.so), 3 runs each interleaved, then a
# rocprofv3 kernel trace of this tree's timer split into kernel duration and launch gap (tools/trace_gaps.py).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-sct}
for i in 1 2 3; do
  timeout -k 10 60 ./build/short_call_timer 2000 > gpurun_out/${tag}_new_$i.json
  timeout -k 10 60 ./build/short_call_timer_ref 2000 > gpurun_out/${tag}_ref_$i.json
done
rm -rf gpurun_out/${tag}_trace
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -- ./build/short_call_timer 2000 > gpurun_out/${tag}_trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/${tag}_trace 2000 > gpurun_out/${tag}_gaps.txt

#!/bin/bash
# IIR A/B (development tool): GPU IIR tests, then gsdrIirFF/CC timing of the in-tree build against the
# builds given as arguments, then per-kernel kernel-trace means of the in-tree build.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_iir.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 200 python tools/iir_time_libs.py "$@" || exit 1
IIR_KINDS="ff cc" bash tools/iir_prof.sh

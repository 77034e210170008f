#!/bin/bash
# Quick tuning session: FIR variant parity, then the variant sweep.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_fir.py -m gpu -q -x -p no:cacheprovider --timeout 300 -k "variants or full_config or parity" > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_sweep.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/fir_probe.py ${PROBE_ARGS} > gpurun_out/probe.log 2>&1; rc=$?
cat gpurun_out/probe.log; exit $rc

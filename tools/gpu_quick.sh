#!/bin/bash
# Quick GPU session: selected tests (PYTEST_K / PYTEST_FILES), then a short bench (development tool).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_quick.log 2>&1; rc=$?
tail -4 gpurun_out/t_quick.log; [ $rc -le 1 ] || exit $rc; [ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-30} ${BENCH_ARGS} > gpurun_out/bench_quick.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1])
print('headline us', d['roofline']['kernel_us_mean'], 'frac', d['roofline']['frac'])
for k, v in d['secondary'].items():
    print(k, {kk: vv for kk, vv in v.items() if 'us' in kk})
PY

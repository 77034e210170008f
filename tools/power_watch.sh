#!/bin/bash
# Run a program while sampling sclk / package power every ~0.3 s (development tool).
mkdir -p gpurun_out
"$@" > gpurun_out/power_prog.log 2>&1 &
pid=$!
: > gpurun_out/power_watch.log
while kill -0 $pid 2>/dev/null; do
  { date +%s.%N; timeout 5 rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Package Power"; } >> gpurun_out/power_watch.log
  sleep 0.1
done
wait $pid; rc=$?
cat gpurun_out/power_prog.log
python3 - <<'PY'
import re
txt = open('gpurun_out/power_watch.log').read()
for b in re.split(r'\n(?=\d{10}\.\d+\n)', txt):
    s = re.findall(r'sclk clock level: \d+: \((\d+)Mhz\)', b); p = re.findall(r'Package Power \(W\): ([\d.]+)', b)
    if s and p: print(b.split('\n')[0][-12:], s[0], 'MHz', p[0], 'W')
PY
exit $rc

#!/bin/bash
# Sample GPU clock/power while a sustained probe runs (development tool).
mkdir -p gpurun_out
python tools/sustained_probe.py $EXTRA --variants "$1" --launches "${2:-6000}" --window 1000 --cool 1 > gpurun_out/clock_probe.log 2>&1 &
pid=$!
for i in $(seq 1 40); do
  { date +%s.%N; timeout 5 rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|fclk|mclk|Power|Temperature|Socket" ; } >> gpurun_out/clock_watch.log
  kill -0 $pid 2>/dev/null || break
  sleep 0.2
done
wait $pid
cat gpurun_out/clock_probe.log

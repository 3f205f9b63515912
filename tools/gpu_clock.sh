#!/bin/bash
# GFX clock and power while the pipeline runs in steady state: a long bench
# (1000 steps) with rocm-smi sampling beside it.
set -o pipefail
O=gpurun_out/clock
mkdir -p $O
(HBX_K1_MODE=${K1MODE:-2} timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1000 > $O/bench.json 2> $O/bench.err; echo "bench rc=$?" >> $O/bench.err) &
BP=$!
for i in $(seq 1 60); do
  date +%s.%N >> $O/smi.log
  timeout 10 rocm-smi --showclocks --showpower --showtemp >> $O/smi.log 2>&1
  kill -0 $BP 2>/dev/null || break
  sleep 0.5
done
wait $BP
cat $O/bench.err | tail -3
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'])"
grep -E "sclk|Power|Temperature \(Sensor (edge|junction)" $O/smi.log | sort | uniq -c | sort -rn | head -40

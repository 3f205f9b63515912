#!/bin/bash
# Round 5 final: the GPU suite and the driver's command with the result push kernel as the default.
set -o pipefail
O=gpurun_out/r05ba
mkdir -p $O
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 240 python bench.py > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench20.json'))
print('bench', d['value'], d.get('check_vs_oracle'), d['host_ms_per_step'], 'zipf', d.get('zipf',{}).get('value'), 'f8?', d['config'].get('workload'))"
timeout -k 10 240 python bench.py --files 8 --steps 20 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime > $O/f8.json 2> $O/f8.err || { tail -20 $O/f8.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/f8.json'))
print('f8', d['value'], d.get('check_vs_oracle'), d['host_ms_per_step']['submit_ms_median_max'], 'zipf', d.get('zipf',{}).get('value'))"

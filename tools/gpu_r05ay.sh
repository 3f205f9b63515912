#!/bin/bash
# Round 5: where the slow submit at step 13 of a 20-step window at 8 files spends its host time (engine phases).
set -o pipefail
O=gpurun_out/r05ay
mkdir -p $O
HBX_TRACE_SLOW_SUBMIT=2 timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime --no-check --workload random --steps 20 --warmup 5 > $O/w5.json 2> $O/w5.err || { tail -20 $O/w5.err; exit 1; }
grep "slow submit" $O/w5.err | tail -20
python3 -c "
import json;d=json.load(open('$O/w5.json'))
print('w5', d['value'], d['host_ms_per_step'])"

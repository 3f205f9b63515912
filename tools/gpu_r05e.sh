#!/bin/bash
# Round 5: plan mode 3 (lag-2 preplan on the cut stream) with K3P: parity
# tests, then the bench A/B on one box (K3P lag 1, K3P lag 2 mode 1 / mode 3,
# shipped K3 lag 1).
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "producer or plan_stream or pipelined" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "1 2 1" "1 2 0" "1 1 0" "0 1 0"; do
  set -- $cfg
  HBX_AB=1 HBX_K3_PROD=$1 HBX_PLAN_CUT=$3 timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --e2e-steps 0 --no-cpu-baseline --join-lag $2 --workload random > $O/bench_p$1_l$2_c$3.json 2> $O/bench_p$1_l$2_c$3.err || { tail -20 $O/bench_p$1_l$2_c$3.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench_p$1_l$2_c$3.json'))
print('prod=$1 lag=$2 cut=$3', d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'], d['lib']['knobs']['plan_mode'])
print(' lifetime', {k: v for k, v in d.get('lifetime', {}).items() if k != 'source'})"
done

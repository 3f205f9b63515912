#!/bin/bash
# Round 5: K3Q without cache-wide fences: parity matrix, then A/B at 64 files.
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "producer" --timeout 120 --timeout-method thread > $O/pytest_k3q.log 2>&1 || { tail -40 $O/pytest_k3q.log; exit 1; }
tail -2 $O/pytest_k3q.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 5 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{})
print('$n', d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'], d['lib']['knobs']['k3_items'], 'cpb', l.get('cycles_per_block'), 'ovh', l.get('launch_overhead'))"
}
BARGS="--steps 100"
run q0 HBX_AB=1 HBX_K3_ITEMS=0 || exit 1
run q4 HBX_AB=1 HBX_K3_ITEMS=4 || exit 1
run q8 HBX_AB=1 HBX_K3_ITEMS=8 || exit 1
run q0b HBX_AB=1 HBX_K3_ITEMS=0 || exit 1
BARGS="--steps 300 --files 8"
run f8_q0 HBX_AB=1 HBX_K3_ITEMS=0 || exit 1
run f8_q2 HBX_AB=1 HBX_K3_ITEMS=2 || exit 1

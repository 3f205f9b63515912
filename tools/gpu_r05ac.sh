#!/bin/bash
# Round 5: plan mode 4 (lag 1, the next launch planned behind each K2r on the cut stream) with K3 period 2 at
# 64 files: same lead as lag 2 / period 1, launch overhead once per 2 steps. Parity, then alternating A/B.
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "period" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS $EXTRA > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs'];c=d['config'];l=d.get('lifetime',{})
print('$n', d['value'], d['check_vs_oracle'], 'lag', c['join_lag'], 'P', c['k3_period'], 'pm', k['plan_mode'], 'B', c['md5_slice_blocks'], 'R', c['pipeline_depth'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'], 'ovh', l.get('launch_overhead'), 'lead', l.get('lead'))"
}
BARGS="--steps 100"
for r in 1 2; do
  EXTRA="" run base_$r || exit 1
  EXTRA="--join-lag 1 --k3-period 2" run m4p2_$r HBX_AB=1 HBX_K2_STREAM=1 HBX_PLAN_CUT=3 || exit 1
done
EXTRA="--join-lag 1 --k3-period 1" run m4p1 HBX_AB=1 HBX_K2_STREAM=1 HBX_PLAN_CUT=3 || exit 1
EXTRA="--join-lag 2 --k3-period 2" run l2p2 || exit 1

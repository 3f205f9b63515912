#!/bin/bash
# Round 5: K3P producer with three register sets in flight (HBX_K3_PSETS=3): parity, then alternating A/B.
set -o pipefail
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -k "producer_waves and (p3 or 1-) or schedule" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'psets', k['k3_psets'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'], 'cpb', l.get('cycles_per_block'), 'ovh', l.get('launch_overhead'))"
}
BARGS="--steps 100"
for r in 1 2 3; do
  run p2_$r HBX_AB=1 HBX_K3_PSETS=2 || exit 1
  run p3_$r HBX_AB=1 HBX_K3_PSETS=3 || exit 1
done
BARGS="--steps 400 --files 8"
run f8_p2 HBX_AB=1 HBX_K3_PSETS=2 || exit 1
run f8_p3 HBX_AB=1 HBX_K3_PSETS=3 || exit 1

#!/bin/bash
# Round 5: side kernels (K2, K2r, plan, K4, meta fetch) padded in LDS so they never share a CU with K3P: parity, A/B.
set -o pipefail
O=gpurun_out/r05ag
mkdir -p $O
HBX_AB=1 HBX_SIDE_PAD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -k "pipelined or period or schedule or mixed" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'pad', k['side_pad'], d['kernel_ms_per_step'], 'cpb', l.get('cycles_per_block'), 'ovh', l.get('launch_overhead'))"
}
BARGS="--steps 100"
for r in 1 2 3; do
  run pad0_$r HBX_AB=1 HBX_SIDE_PAD=0 || exit 1
  run pad1_$r HBX_AB=1 HBX_SIDE_PAD=1 || exit 1
done
BARGS="--steps 400 --files 8"
run f8_pad0 HBX_AB=1 HBX_SIDE_PAD=0 || exit 1
run f8_pad1 HBX_AB=1 HBX_SIDE_PAD=1 || exit 1

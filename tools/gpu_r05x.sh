#!/bin/bash
# Round 5: K1 tail tiles (short tiles after the long ones): parity, then alternating A/B at 8, 16 and 64 files.
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "tail_tiles or tile_sizes" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'tail', k['k1_tail'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
BARGS="--steps 400 --files 8"
for r in 1 2; do
  run f8_t0_$r HBX_AB=1 HBX_K1_TAIL=0 || exit 1
  run f8_t1_$r HBX_AB=1 HBX_K1_TAIL=1 || exit 1
done
BARGS="--steps 200 --files 16"
run f16_t0 HBX_AB=1 HBX_K1_TAIL=0 || exit 1
run f16_t1 HBX_AB=1 HBX_K1_TAIL=1 || exit 1
BARGS="--steps 100"
for r in 1 2; do
  run f64_t0_$r HBX_AB=1 HBX_K1_TAIL=0 || exit 1
  run f64_t1_$r HBX_AB=1 HBX_K1_TAIL=1 || exit 1
done

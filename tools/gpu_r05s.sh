#!/bin/bash
# Round 5: alternating A/B of K1 tile length at 8 files per GPU (16 / 24 / 28 iterations, three rounds).
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime --no-check $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], 'tile', k['tile_iters'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
BARGS="--steps 400 --files 8"
for r in 1 2 3; do
  run t16_$r HBX_AB=1 HBX_TILE_ITERS=16 || exit 1
  run t24_$r HBX_AB=1 HBX_TILE_ITERS=24 || exit 1
  run t28_$r HBX_AB=1 HBX_TILE_ITERS=28 || exit 1
done

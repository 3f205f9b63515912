#!/bin/bash
# Round 5: K1 tile length sweep, 8 / 16 / 32 files per GPU (HBX_TILE_ITERS).
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'tile', k['tile_iters'], 'P', c['k3_period'], d['kernel_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
run f8_t20 HBX_AB=1 HBX_TILE_ITERS=20 || exit 1
run f8_t24 HBX_AB=1 HBX_TILE_ITERS=24 || exit 1
run f8_t28 HBX_AB=1 HBX_TILE_ITERS=28 || exit 1
run f8_t16 HBX_AB=1 HBX_TILE_ITERS=16 || exit 1
BARGS="--steps 200 --files 16"
run f16_t32 HBX_AB=1 HBX_TILE_ITERS=32 || exit 1
run f16_t48 HBX_AB=1 HBX_TILE_ITERS=48 || exit 1
run f16_t64 HBX_AB=1 HBX_TILE_ITERS=64 || exit 1
BARGS="--steps 200 --files 32"
run f32_t64 HBX_AB=1 HBX_TILE_ITERS=64 || exit 1
run f32_t96 HBX_AB=1 HBX_TILE_ITERS=96 || exit 1
run f32_t128 HBX_AB=1 HBX_TILE_ITERS=128 || exit 1

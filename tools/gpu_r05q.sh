#!/bin/bash
# Round 5: K1 tile length at 8 files per GPU with the K3 period (HBX_TILE_ITERS sweep).
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'tile', k['tile_iters'], 'P', c['k3_period'], d['kernel_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
run t16 HBX_AB=1 HBX_TILE_ITERS=16 || exit 1
run t24 HBX_AB=1 HBX_TILE_ITERS=24 || exit 1
run t32 HBX_AB=1 HBX_TILE_ITERS=32 || exit 1
run t12 HBX_AB=1 HBX_TILE_ITERS=12 || exit 1
run t64 HBX_AB=1 HBX_TILE_ITERS=64 || exit 1
run t16b HBX_AB=1 HBX_TILE_ITERS=16 || exit 1
run t24b HBX_AB=1 HBX_TILE_ITERS=24 || exit 1

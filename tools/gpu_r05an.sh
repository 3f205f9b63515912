#!/bin/bash
# Round 5: K3 grid of 128 workgroups (just above the ~124 busy ones) vs one per CU (256).
set -o pipefail
O=gpurun_out/r05an
mkdir -p $O
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'wgs', k['md5_wgs'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
BARGS="--steps 100"
for r in 1 2; do
  run w256_$r HBX_AB=1 || exit 1
  run w128_$r HBX_AB=1 HBX_K3_WGS=128 || exit 1
done
BARGS="--steps 400 --files 8"
run f8_w256 HBX_AB=1 || exit 1
run f8_w128 HBX_AB=1 HBX_K3_WGS=128 || exit 1

#!/bin/bash
# Round 5: join lag 2 vs 3 at 32 and 16 files per GPU (alternating).
set -o pipefail
O=gpurun_out/r05ak
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime --no-check "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', d['value'], 'P', c['k3_period'], 'lag', c['join_lag'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
for r in 1 2; do
  run f32_l3_$r --files 32 --steps 200 || exit 1
  run f32_l2_$r --files 32 --steps 200 --join-lag 2 || exit 1
done
for r in 1 2; do
  run f16_l3_$r --files 16 --steps 200 || exit 1
  run f16_l2_$r --files 16 --steps 200 --join-lag 2 || exit 1
done

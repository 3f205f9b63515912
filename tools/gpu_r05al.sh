#!/bin/bash
# Round 5: join lag 2 vs 3 at 8 files per GPU (alternating, three pairs).
set -o pipefail
O=gpurun_out/r05al
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime --no-check "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));c=d['config'];print('$n', d['value'], 'P', c['k3_period'], 'lag', c['join_lag'], 'R', c['pipeline_depth'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
for r in 1 2 3; do
  run f8_l3_$r --files 8 --steps 400 || exit 1
  run f8_l2_$r --files 8 --steps 400 --join-lag 2 || exit 1
done

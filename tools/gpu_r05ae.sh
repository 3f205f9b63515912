#!/bin/bash
# Round 5: arenas as R allocations vs views of one allocation (translation reach of K3's scattered chains).
set -o pipefail
O=gpurun_out/r05ae
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-check $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{})
print('$n', d['value'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'], 'cpb', l.get('cycles_per_block'), 'ovh', l.get('launch_overhead'))"
}
BARGS="--steps 100"
for r in 1 2; do
  run sep_$r || exit 1
  run one_$r --single-alloc || exit 1
done

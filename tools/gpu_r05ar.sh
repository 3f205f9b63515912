#!/bin/bash
# Round 5: which step of a 20-step window at 8 files per GPU holds the one slow submit, and whether it moves
# with the warm-up length (a fixed absolute submit count) or not (a fixed place after the pre-window sync).
set -o pipefail
O=gpurun_out/r05ar
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime --no-check --workload random "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d['host_ms_per_step'], d['config'].get('resident_batches'))"
}
run w5 --steps 20 --warmup 5 || exit 1
run w8 --steps 20 --warmup 8 || exit 1
run w12 --steps 20 --warmup 12 || exit 1
run w20 --steps 20 --warmup 20 || exit 1
run p1w5 --steps 20 --warmup 5 --k3-period 1 || exit 1

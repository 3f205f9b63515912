#!/bin/bash
# Round 5: why a 20-step window's first leg at 8 files per GPU runs slow (host submit time per step), and
# whether a longer warm-up cures it.
set -o pipefail
O=gpurun_out/r05ap
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d['host_ms_per_step'], 'zipf', d.get('zipf',{}).get('value'), d.get('zipf',{}).get('host_ms_per_step'))"
}
run w5 --steps 20 --warmup 5 || exit 1
run w5b --steps 20 --warmup 5 || exit 1
run w40 --steps 20 --warmup 40 || exit 1
run s200 --steps 200 --warmup 5 --workload random || exit 1

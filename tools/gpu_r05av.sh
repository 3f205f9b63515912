#!/bin/bash
# Round 5: the slow submit at step 13 of a 20-step window at 8 files: the GPU-side fence or the submit call?
set -o pipefail
O=gpurun_out/r05av
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime --no-check --workload random "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d['host_ms_per_step'])"
}
run w5 --steps 20 --warmup 5 || exit 1

MALLOC_MMAP_THRESHOLD_=1048576 run w5mmap --steps 20 --warmup 5 || exit 1

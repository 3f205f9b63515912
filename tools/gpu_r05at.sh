#!/bin/bash
# Round 5: the slow submit at step 13 of a 20-step window at 8 files: does it move with HIP's hardware-queue count
# or AQL queue size (streams sharing a queue / a full queue), or with the join lag?
set -o pipefail
O=gpurun_out/r05at
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime --no-check --workload random "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d['host_ms_per_step'])"
}
run w5 --steps 20 --warmup 5 || exit 1
GPU_MAX_HW_QUEUES=8 run w5hwq8 --steps 20 --warmup 5 || exit 1
ROC_AQL_QUEUE_SIZE=65536 run w5aql64k --steps 20 --warmup 5 || exit 1
run w5s40 --steps 40 --warmup 5 || exit 1
run w5lag3 --steps 20 --warmup 5 --join-lag 3 || exit 1

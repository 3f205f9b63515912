#!/bin/bash
# Per-GPU throughput at the strong-scaling batch sizes (files per GPU = 64/N):
# join lag 1 vs 2; at lag 2 the plan inline on the scan stream (HBX_PLAN_MODE=0),
# on the hash stream (1) or one launch ahead (default).
set -o pipefail
out=gpurun_out/lag
mkdir -p $out
for nf in ${@:-8 16 32 64}; do
  for cfg in "1 -" "2 0" "2 1" "2 -"; do
    set -- $cfg
    tag=nf${nf}_lag$1_plan$2
    if [ "$2" = "-" ]; then unset HBX_PLAN_MODE; else export HBX_PLAN_MODE=$2; fi
    timeout -k 10 240 python bench.py \
      --no-cpu-baseline --no-check --workload random --steps 200 --files $nf --join-lag $1 \
      > $out/$tag.json 2> $out/$tag.err || exit 1
    python - $out/$tag.json $tag <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernel_ms_per_step"]
print(f"{sys.argv[2]} R={d['config']['pipeline_depth']} B={d['config']['md5_slice_blocks']} "
      f"{d['value']:.1f} GiB/s {d['ms_per_step']:.3f} ms  " + " ".join(f"{n}={v:.3f}" for n,v in k.items()), flush=True)
PY
  done
done

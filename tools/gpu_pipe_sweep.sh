#!/bin/bash
# Per-GPU pipeline sweep: each argument is "files:lag:lead" (lead "-" = the
# default; the plan placement follows the lag).  Prints value, ms/step and
# kernel ms/step.
# usage: bash tools/gpu_pipe_sweep.sh 8:2:- 8:3:6 ...
set -o pipefail
out=gpurun_out/pipe
mkdir -p $out
for cfg in "$@"; do
  IFS=: read nf lag lead <<< "$cfg"
  la=""; [ "$lead" != "-" ] && la="--lead $lead"
  tag=nf${nf}_lag${lag}_l${lead}
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-check --workload random --steps 200 \
    --files $nf --join-lag $lag $la > $out/$tag.json 2> $out/$tag.err || { tail -3 $out/$tag.err; exit 1; }
  python - $out/$tag.json $tag <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernel_ms_per_step"]; c=d["config"]; h=d.get("host_ms_per_step", {})
print(f"{sys.argv[2]:24s} R={c['pipeline_depth']} B={c['md5_slice_blocks']} lead={c['scan_lead']} "
      f"{d['value']:.1f} GiB/s {d['ms_per_step']:.3f} ms  host sub {h.get('submit_ms',0):.3f} col {h.get('collect_ms',0):.3f} (wait {h.get('in_hbx_wait_ms',0):.3f})  " + " ".join(f"{n[:6]}={v:.3f}" for n,v in k.items()), flush=True)
PY
done

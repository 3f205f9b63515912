#!/bin/bash
# K3P's per-wave launch timeline inside the bench schedule (--k3-probe).
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
HBX_AB=1 HBX_K3_PROD=1 timeout -k 10 300 python bench.py --gpus 1 --steps 40 --warmup 5 --e2e-steps 0 --no-cpu-baseline --k3-probe --workload random > $O/probe_p1.json 2> $O/probe_p1.err || { tail -20 $O/probe_p1.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/probe_p1.json'))
print(d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'])
print(' lifetime', {k: v for k, v in d.get('lifetime', {}).items() if k != 'source'})
p=d.get('k3_probe'); print(' probe', p)"

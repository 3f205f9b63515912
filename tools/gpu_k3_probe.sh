#!/bin/bash
# Per-wave timeline of one steady-state K3 launch (bench.py --k3-probe) at the given batch sizes.
set -o pipefail
for nf in ${@:-8 64}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --workload random --steps 50 --files $nf --k3-probe --e2e-steps 0 \
    > gpurun_out/probe_$nf.json 2> gpurun_out/probe.err || { tail -3 gpurun_out/probe.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/probe_$nf.json').read().strip().splitlines()[-1]);print($nf, d['value'], d['kernel_ms_per_step']['k3_block_md5'], json.dumps(d['k3_probe']))"
done

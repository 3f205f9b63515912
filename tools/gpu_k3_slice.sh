#!/bin/bash
# K3 launch time vs slice B at a fixed residency (8 files per GPU, 256 batches): the per-launch fixed cost.
set -o pipefail
for B in 521 1042 2084 4168; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --workload random --steps 100 --files 8 --arenas 256 --md5-slice $B > gpurun_out/k3c_$B.json 2> gpurun_out/k3c_$B.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/k3c_$B.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print($B, d['value'], d['ms_per_step'], k['k3_block_md5'], k['k1_digest_scan'])"
done

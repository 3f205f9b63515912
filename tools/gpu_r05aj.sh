#!/bin/bash
# Round 5 final tree: one GPU's share of configs[2] at N = 2, 4, 8 (32, 16, 8 files per step), bench defaults.
set -o pipefail
O=gpurun_out/r05aj
mkdir -p $O
for f in 32 16 8; do
  timeout -k 10 300 python bench.py --gpus 1 --files $f --steps 200 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random > $O/f$f.json 2> $O/f$f.err || { tail -20 $O/f$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f$f.json'));c=d['config'];print('$f files', d['value'], d['fill_drain_gibs'], d['check_vs_oracle'], 'P', c['k3_period'], 'lag', c['join_lag'], 'R', c['pipeline_depth'], 'B', c['md5_slice_blocks'], d['kernel_ms_per_step'])"
done

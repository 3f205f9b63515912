#!/bin/bash
# A/B: scan lead (how many steps K1/K2 run ahead of K3) on the current build
set -o pipefail
O=gpurun_out
for l in 2 3 2 3 4; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --lead $l > $O/ld_$l.json 2> $O/ld_$l.err || { tail -5 $O/ld_$l.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ld_$l.json'));print('$l', d['value'], d['config']['pipeline_depth'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'])"
done

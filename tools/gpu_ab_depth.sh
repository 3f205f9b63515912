#!/bin/bash
# A/B: resident batches (pipeline depth) on the current build
set -o pipefail
O=gpurun_out
for r in auto 34 auto 34 32; do
  if [ $r = auto ]; then A=""; else A="--arenas $r"; fi
  timeout -k 10 180 python bench.py --no-cpu-baseline $A > $O/dp_$r.json 2> $O/dp_$r.err || { tail -5 $O/dp_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dp_$r.json'));print('$r', d['value'], d['config']['pipeline_depth'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'])"
done

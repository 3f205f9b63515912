#!/bin/bash
# A/B: K2 on a stream of its own (HBX_K2_STREAM=1) beside the masked scan stream
set -o pipefail
O=gpurun_out
for v in 0 1 0 1; do
  HBX_K2_STREAM=$v timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/k2s_$v.json 2> $O/k2s_$v.err || { tail -5 $O/k2s_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/k2s_$v.json'));print('$v', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
done

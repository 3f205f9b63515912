#!/bin/bash
# A/B: K1 variants (0 VGPR loads, 1 DMA into LDS (default), 2 lite) on the power-capped pipeline
set -o pipefail
O=gpurun_out
for m in 1 0 2 1 0 2; do
  HBX_K1_MODE=$m timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/k1m_$m.json 2> $O/k1m_$m.err || { tail -5 $O/k1m_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/k1m_$m.json'));print('$m', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
done

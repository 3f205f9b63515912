#!/bin/bash
# A/B: K1 tile size beside K3 (smaller tiles free CUs for the next K3 launch sooner)
set -o pipefail
O=gpurun_out
for t in ${TILES:-64 16 32 8 64 16}; do
  HBX_TILE_ITERS=$t timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/ti_$t.json 2> $O/ti_$t.err || { tail -5 $O/ti_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ti_$t.json'));print('tile_iters $t', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
done

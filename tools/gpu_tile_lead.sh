#!/bin/bash
# K1 tile length vs the scan lead: does a finer K1 tile (more, shorter
# rounds over the CUs K3 leaves) remove the lead-1 cliff?
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/${TAG:-tile_lead}
mkdir -p $O
for cfg in "64 1" "128 1" "32 1" "16 1" "128 -1"; do
  set -- $cfg
  timeout -k 10 240 env HBX_TILE_ITERS=$1 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check --lead $2 > $O/t$1_l$2.json 2> $O/t$1_l$2.err || { tail -20 $O/t$1_l$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t$1_l$2.json'));print('tile $1 lead $2', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['config']['md5_slice_blocks'], d['k3_lanes']['active_chains_mean'])"
done

#!/bin/bash
# Strong-scaling batch (8 files per GPU, the N = 8 share): K1 vs K1b and the
# K1 tile length, alternating.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/${TAG:-small_k1}; mkdir -p $O
for i in 1 2; do for cfg in "64 0" "128 0" "64 16" "128 16"; do
  set -- $cfg
  timeout -k 10 240 env HBX_K1_RUN=$1 HBX_TILE_ITERS=$2 python bench.py --files 8 --steps 200 --warmup 5 --workload random --no-cpu-baseline --no-check > $O/r$1_t$2_$i.json 2> $O/r$1_t$2_$i.err || { tail -20 $O/r$1_t$2_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r$1_t$2_$i.json'));print('run $1 tile $2 #$i', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done; done

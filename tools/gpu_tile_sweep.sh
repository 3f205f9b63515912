#!/bin/bash
# K1 tile length per batch size (files per GPU = 64/N of strong scaling):
# the automatic choice (two tiles per CU) vs shorter tiles, alternating.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/${TAG:-tile_sweep}; mkdir -p $O
for cfg in ${CFGS:-"8 8" "8 16" "16 0" "16 16" "16 32" "32 0" "32 32" "32 64" "64 0" "64 128" "8 0"}; do
  set -- $cfg
  timeout -k 10 240 env HBX_TILE_ITERS=$2 python bench.py --files $1 --steps 200 --warmup 5 --workload random --no-cpu-baseline --no-check > $O/f$1_t$2.json 2> $O/f$1_t$2.err || { tail -20 $O/f$1_t$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f$1_t$2.json'));print('files $1 tile $2', d['value'], d['ms_per_step'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
done

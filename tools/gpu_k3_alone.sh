#!/bin/bash
# K3 per-launch time with K1 serialized against it (CU-masked hash stream, every CU set):
# separates K3's in-kernel fixed cost from K1's interference.  usage: bash tools/gpu_k3_alone.sh [files...]
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
for nf in ${@:-8 64}; do
  for m in "" "0:4096"; do
    HBX_HASH_CUS=$m timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --workload random --steps 100 --files $nf \
      > gpurun_out/k3alone_${nf}_${m:-none}.json 2> gpurun_out/k3alone.err || { tail -3 gpurun_out/k3alone.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/k3alone_${nf}_${m:-none}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; c=d['config']
print('files=$nf hash_cus=${m:-none}', 'B', c['md5_slice_blocks'], d['value'], d['ms_per_step'], 'K3', k['k3_block_md5'], 'K1', k['k1_digest_scan'])"
  done
done

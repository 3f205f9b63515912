#!/bin/bash
# K1 tiles fitted to the CUs K3 leaves (default) vs two per CU (HBX_K1_FIT=0),
# at 33-36 resident batches (64 files) and at strong-scaling batch sizes.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
out=gpurun_out/k1fit; mkdir -p $out
run() {  # tag fit args...
  local tag=$1 fit=$2; shift 2
  HBX_K1_FIT=$fit timeout -k 10 240 python bench.py --no-cpu-baseline --no-check --workload random --steps 200 "$@" \
    > $out/$tag.json 2> $out/$tag.err || { tail -3 $out/$tag.err; exit 1; }
  python - $out/$tag.json $tag <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernel_ms_per_step"]; c=d["config"]
print(f"{sys.argv[2]:18s} files={c['files_per_gpu']} R={c['pipeline_depth']} B={c['md5_slice_blocks']} {d['value']:.1f} GiB/s "
      f"{d['ms_per_step']:.3f} ms  K1 {k['k1_digest_scan']:.3f} K3 {k['k3_block_md5']:.3f} active {d['k3_lanes']['active_chains_mean'] if d['k3_lanes'] else None}", flush=True)
PY
}
for R in ${ARENAS:-33 34 35}; do
  run fit1_R$R 1 --arenas $R
  run fit0_R$R 0 --arenas $R
done
for nf in ${FILES:-8 16}; do
  run fit1_nf$nf 1 --files $nf
  run fit0_nf$nf 0 --files $nf
done

#!/bin/bash
# Round 5: CU split at 8 files per GPU: fewer resident batches (hbm-frac) put fewer chains in flight, so K3
# takes fewer CUs and K1 more; plus the new period cases of the verify / store_paths tests.
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py tests/test_gpu_parity.py -x -v -k "pipelined_verify or store_paths_end" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));c=d['config']
print('$n', d['value'], d['check_vs_oracle'], 'R', c['pipeline_depth'], 'B', c['md5_slice_blocks'], 'lanes', d['k3_lanes']['active_chains_mean'] if d.get('k3_lanes') else None, d['kernel_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
run h95 --hbm-frac 0.95 || exit 1
run h90 --hbm-frac 0.90 || exit 1
run h86 --hbm-frac 0.86 || exit 1
run h82 --hbm-frac 0.82 || exit 1
run h78 --hbm-frac 0.78 || exit 1
run h95b --hbm-frac 0.95 || exit 1
run h86b --hbm-frac 0.86 || exit 1

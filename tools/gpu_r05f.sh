#!/bin/bash
# Round 5: shipped K3 (lag 1) vs K3P + plan mode 3 (lag 2), alternating twice at
# 200 steps on one box; then the N = 8 strong-scaling share (8 files per GPU,
# lag 3) with and without K3P.
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-lifetime --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'], d['lib']['knobs']['plan_mode'], d['lib']['knobs']['k3_prod'])"
}
BARGS="--steps 200"
for rep in 1 2; do
  run base_$rep HBX_AB=1 HBX_K3_PROD=0 || exit 1
  BARGS="--steps 200 --join-lag 2" run k3p_m3_$rep HBX_AB=1 HBX_K3_PROD=1 HBX_PLAN_CUT=1 || exit 1
done
BARGS="--steps 400 --files 8"
run base_f8 HBX_AB=1 HBX_K3_PROD=0 || exit 1
run k3p_f8 HBX_AB=1 HBX_K3_PROD=1 || exit 1

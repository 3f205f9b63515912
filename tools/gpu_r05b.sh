#!/bin/bash
# Round 5: K3 floors (tools/ubench/k3_prod: LDS-fed and register-only MD5
# waves) and the per-wave K3 timeline (--k3-probe) of the shipped K3 and K3P
# inside the bench schedule, with the steady-state lifetime decomposition.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 240 tools/ubench/k3_prod 64 32768 4096 3 > $O/k3_prod.txt 2>&1; rc=$?
cat $O/k3_prod.txt
[ $rc -eq 0 ] || exit $rc
for cfg in "1 2" "0 1"; do
  set -- $cfg
  HBX_AB=1 HBX_K3_PROD=$1 timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --e2e-steps 0 --no-cpu-baseline --join-lag $2 --k3-probe --workload random > $O/probe_p$1_l$2.json 2> $O/probe_p$1_l$2.err || { tail -20 $O/probe_p$1_l$2.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/probe_p$1_l$2.json'))
print('prod=$1 lag=$2', d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'])
print(' lifetime', d.get('lifetime'))
p=d.get('k3_probe'); print(' probe', {k: p[k] for k in p if k not in ('slowest10',)})"
done

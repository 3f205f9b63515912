#!/bin/bash
# Round 5: K3P with hand-placed LDS waits in the MD5 wave (k3p_consume):
# ubench floors, the K3/K3P parity tests, and the bench A/B on one box.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 240 tools/ubench/k3_prod 64 32768 4096 3 > $O/k3_prod.txt 2>&1; rc=$?
cat $O/k3_prod.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "producer" --timeout 120 --timeout-method thread > $O/pytest_k3p.log 2>&1 || { tail -30 $O/pytest_k3p.log; exit 1; }
tail -2 $O/pytest_k3p.log
for cfg in "1 1" "1 2" "0 1"; do
  set -- $cfg
  HBX_AB=1 HBX_K3_PROD=$1 timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 --e2e-steps 0 --no-cpu-baseline --join-lag $2 --workload random > $O/bench_p$1_l$2.json 2> $O/bench_p$1_l$2.err || { tail -20 $O/bench_p$1_l$2.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench_p$1_l$2.json'))
print('prod=$1 lag=$2', d['value'], d['check_vs_oracle'], d['kernel_ms_per_step'])
print(' lifetime', {k: v for k, v in d.get('lifetime', {}).items() if k != 'source'})"
done

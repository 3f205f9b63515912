#!/bin/bash
# Round 5: finalizations deferred to the end of a submit + lean K1 timing with K2 on the cut stream: parity, A/B.
set -o pipefail
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_verify.py -x -v -k "period or pipelined or input_after or fence or schedule or plan_stream or reserved" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'defer', k['defer_fin'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'], d['host_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
for r in 1 2; do
  run f8_d0_$r HBX_AB=1 HBX_DEFER_FIN=0 || exit 1
  run f8_d1_$r HBX_AB=1 HBX_DEFER_FIN=1 || exit 1
done
BARGS="--steps 100"
for r in 1 2; do
  run f64_d0_$r HBX_AB=1 HBX_DEFER_FIN=0 || exit 1
  run f64_d1_$r HBX_AB=1 HBX_DEFER_FIN=1 || exit 1
done

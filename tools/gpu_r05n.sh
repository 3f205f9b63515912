#!/bin/bash
# Round 5: 8 files per GPU, K3 period 4: scan lead (lag + P vs lag + 1 vs lag + 2P), then 16 / 32 files.
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_abi.py tests/test_gpu_fullsize.py -x -v -k "knob or ab or schedule" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'P', c['k3_period'], 'lead', c['scan_lead'], 'B', c['md5_slice_blocks'], 'pm', k['plan_mode'], d['kernel_ms_per_step'], 'host', d['host_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
run f8_auto || exit 1
run f8_l4 --lead 4 || exit 1
run f8_l11 --lead 11 || exit 1
run f8_autob || exit 1
run f8_p2 --k3-period 2 || exit 1
run f8_p8 --k3-period 8 || exit 1
BARGS="--steps 200 --files 16"
run f16_auto || exit 1
BARGS="--steps 200 --files 32"
run f32_p1 --k3-period 1 || exit 1
run f32_auto || exit 1

#!/bin/bash
# Round 5: K3 completion events in a launch-indexed ring of 16: parity, then lead / period A/B at 8-32 files.
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -x -v -k "period or pipelined or input_after or fence or reserved or knob or plan_stream" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'P', c['k3_period'], 'lead', c['scan_lead'], 'B', c['md5_slice_blocks'], d['kernel_ms_per_step'], 'collect', d['host_ms_per_step']['collect_ms'])"
}
BARGS="--steps 400 --files 8"
run f8_p8_l11 || exit 1
run f8_p8_l4 --lead 4 || exit 1
run f8_p4_l7 --k3-period 4 || exit 1
run f8_p4_l4 --k3-period 4 --lead 4 || exit 1
run f8_p8_l11b || exit 1
BARGS="--steps 200 --files 16"
run f16_p4_l7 || exit 1
run f16_p4_l4 --lead 4 || exit 1
run f16_p2_l5 --k3-period 2 || exit 1
BARGS="--steps 200 --files 32"
run f32_p2_l5 || exit 1
run f32_p1 --k3-period 1 || exit 1

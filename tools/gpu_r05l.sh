#!/bin/bash
# Round 5: batch meta by kernel (hbx_meta_fetch) and the lag-3 preplan on the cut stream: parity, A/B.
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -k "period or pipelined or producer_waves or input_after or fence or schedule or configs1" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'P', c['k3_period'], 'mk', k['meta_kernel'], 'pm', k['plan_mode'], d['kernel_ms_per_step'], 'ovh', l.get('launch_overhead'))"
}
BARGS="--steps 400 --files 8 --k3-period 4"
run f8_m0 HBX_AB=1 HBX_META_KERNEL=0 || exit 1
run f8_m1 HBX_AB=1 HBX_META_KERNEL=1 || exit 1
run f8_m1c2 HBX_AB=1 HBX_META_KERNEL=1 HBX_PLAN_CUT=2 || exit 1
run f8_m0b HBX_AB=1 HBX_META_KERNEL=0 || exit 1
run f8_m1b HBX_AB=1 HBX_META_KERNEL=1 || exit 1
run f8_m1c2b HBX_AB=1 HBX_META_KERNEL=1 HBX_PLAN_CUT=2 || exit 1
BARGS="--steps 100"
run f64_m0 HBX_AB=1 HBX_META_KERNEL=0 || exit 1
run f64_m1 HBX_AB=1 HBX_META_KERNEL=1 || exit 1
run f64_m0b HBX_AB=1 HBX_META_KERNEL=0 || exit 1
run f64_m1b HBX_AB=1 HBX_META_KERNEL=1 || exit 1

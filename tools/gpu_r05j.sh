#!/bin/bash
# Round 5: K3 period (one K3 launch every P submits): parity, then 8 files per GPU A/B over P.
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -k "period or pipelined or input_after or input_fence or producer_waves and 4096-2" --timeout 120 --timeout-method thread > $O/pytest_period.log 2>&1 || { tail -40 $O/pytest_period.log; exit 1; }
tail -2 $O/pytest_period.log
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));l=d.get('lifetime',{});c=d['config']
print('$n', d['value'], d['check_vs_oracle'], 'P', c['k3_period'], 'B', c['md5_slice_blocks'], 'R', c['pipeline_depth'], d['kernel_ms_per_step'], 'launch', d['roofline']['avg_launch_ms'], 'ovh', l.get('launch_overhead'), 'cpb', l.get('cycles_per_block'))"
}
BARGS="--steps 400 --files 8"
run f8_p1 --k3-period 1 || exit 1
run f8_p2 --k3-period 2 || exit 1
run f8_p4 --k3-period 4 || exit 1
run f8_p8 --k3-period 8 || exit 1
run f8_p1b --k3-period 1 || exit 1
run f8_p4b --k3-period 4 || exit 1
BARGS="--steps 200 --files 16"
run f16_p1 --k3-period 1 || exit 1
run f16_p4 --k3-period 4 || exit 1
BARGS="--steps 100"
run f64_p1 --k3-period 1 || exit 1
run f64_p2 --k3-period 2 || exit 1

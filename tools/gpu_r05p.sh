#!/bin/bash
# Round 5: K1 look-back exchange (no barrier per iteration): parity, then A/B at 64 and 8 files.
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -k "tile or edge or literal or constant or periodic or zipf or mixed or golden or schedule or configs1 or steady" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));c=d['config'];k=d['lib']['knobs']
print('$n', d['value'], d['check_vs_oracle'], 'lb', k['k1_lb'], 'P', c['k3_period'], d['kernel_ms_per_step'])"
}
BARGS="--steps 100"
run f64_lb0 HBX_AB=1 HBX_K1_LB=0 || exit 1
run f64_lb1 HBX_AB=1 HBX_K1_LB=1 || exit 1
run f64_lb0b HBX_AB=1 HBX_K1_LB=0 || exit 1
run f64_lb1b HBX_AB=1 HBX_K1_LB=1 || exit 1
BARGS="--steps 400 --files 8"
run f8_lb0 HBX_AB=1 HBX_K1_LB=0 || exit 1
run f8_lb1 HBX_AB=1 HBX_K1_LB=1 || exit 1
run f8_lb0b HBX_AB=1 HBX_K1_LB=0 || exit 1
run f8_lb1b HBX_AB=1 HBX_K1_LB=1 || exit 1

#!/bin/bash
# Round 5: tile sizing 8/3 per CU up to 2 GiB: parity subset, shares at 8 and 16 files, driver's command.
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -x -v -k "tile or pipelined or period or mixed or edge or schedule or torchrun" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random $BARGS "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));c=d['config']
print('$n', d['value'], d['fill_drain_gibs'], d['check_vs_oracle'], 'P', c['k3_period'], d['kernel_ms_per_step'])"
}
BARGS="--steps 400 --files 8"
run f8 || exit 1
run f8_p1 --k3-period 1 || exit 1
BARGS="--steps 200 --files 16"
run f16 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print('bench20', d['value'], d['fill_drain_gibs'], d['zipf']['value'], d['check_vs_oracle'], d['zipf']['check_vs_oracle'], d['roofline']['frac'], 'e2e', d.get('e2e',{}).get('value'))"

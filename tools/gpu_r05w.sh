#!/bin/bash
# Round 5: K1 gate A/B at 8 and 64 files (alternating), the --e2e headline at 8 files, meta fetch parity.
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "period or tile or pipelined_batches" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --warmup 8 --e2e-steps 0 --no-cpu-baseline --workload random --no-lifetime --no-check $BARGS > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'));k=d['lib']['knobs']
print('$n', d['value'], 'gate', k['k1_gate'], d['kernel_ms_per_step']['k1_digest_scan'], d['kernel_ms_per_step']['k3_block_md5'])"
}
BARGS="--steps 400 --files 8"
for r in 1 2; do
  run f8_g1_$r HBX_AB=1 HBX_K1_GATE=1 || exit 1
  run f8_g0_$r HBX_AB=1 HBX_K1_GATE=0 || exit 1
done
BARGS="--steps 100"
for r in 1 2; do
  run f64_g1_$r HBX_AB=1 HBX_K1_GATE=1 || exit 1
  run f64_g0_$r HBX_AB=1 HBX_K1_GATE=0 || exit 1
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 3 --files 8 --e2e --no-cpu-baseline > $O/e2e_f8.json 2> $O/e2e_f8.err || { tail -20 $O/e2e_f8.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e_f8.json'));print('e2e f8', d['value'], d['check_vs_oracle'], d['config']['k3_period'])"

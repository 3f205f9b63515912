#!/bin/bash
# K3 two waves per SIMD: parity (the parametrized pipelined tests and the
# full-size configs[1] schedule), then the bench at the default residency with
# 1 and 2 waves per SIMD, and the aliased residency sweep with 2.
set -o pipefail
O=gpurun_out/${TAG:-k3w2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "k3_waves or abi" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for W in 1 2; do
  timeout -k 10 240 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --k3-waves $W > $O/bench_w$W.json 2> $O/bench_w$W.err || { tail -20 $O/bench_w$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_w$W.json'));print('w$W', d['value'], d['ms_per_step'], d.get('check_vs_oracle'), d['kernel_ms_per_step'], d['k3_lanes']['active_chains_mean'])"
done
for D in ${DEPTHS:-40 48 56 66}; do
  timeout -k 10 240 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check \
      --hbm-frac 0.85 --alias-depth $D --k3-waves 2 > $O/alias_$D.json 2> $O/alias_$D.err || { tail -20 $O/alias_$D.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/alias_$D.json'));print($D, d['value'], d['ms_per_step'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'], d['k3_lanes']['active_chains_mean'])"
done

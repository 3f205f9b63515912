#!/bin/bash
set -o pipefail
O=gpurun_out
HBX_K1_MODE=2 timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_lite.log 2>&1 || { tail -40 $O/pytest_lite.log; exit 1; }
tail -1 $O/pytest_lite.log
for m in 1 2; do
  HBX_K1_MODE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --check > $O/k1m_$m.json 2> $O/k1m_$m.err || { tail -5 $O/k1m_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/k1m_$m.json'));print('k1 mode $m', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['single_batch']['stages_ms'], d.get('check_vs_oracle'))"
done

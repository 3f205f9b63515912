#!/bin/bash
# parity suite + default bench with the masked scan stream, A/B against HBX_SCAN_CUS=off
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for v in on off on off; do
  if [ $v = off ]; then export HBX_SCAN_CUS=off; else unset HBX_SCAN_CUS; fi
  timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/sm_$v.json 2> $O/sm_$v.err || { tail -5 $O/sm_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sm_$v.json'));print('$v', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
done
unset HBX_SCAN_CUS
timeout -k 10 200 python tools/bench_verify.py > $O/sm_verify.json 2> $O/sm_verify.err || { tail -5 $O/sm_verify.err; exit 1; }
tail -2 $O/sm_verify.json

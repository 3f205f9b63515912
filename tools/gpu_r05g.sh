#!/bin/bash
# Round 5: the whole GPU suite on the new defaults (K3P, plan mode 3, lag 2 at
# 64 files), smoke, and the driver's bench command.
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
grep -E "PASSED|FAILED" $O/pytest_gpu.log | grep -E "hundred|status|producer" | head -40
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'], d['zipf']['value'], d['check_vs_oracle'], d['zipf']['check_vs_oracle'], d['roofline']['frac'], d['valu_roofline'].get('k3'), d['valu_roofline'].get('k1'), 'e2e', d.get('e2e',{}).get('value'), d['cpu_baseline']['value'], d.get('lifetime'))"
timeout -k 10 300 python tools/diag_slow_cu.py --steps 30 > $O/slow_cu.txt 2>&1 || { tail -20 $O/slow_cu.txt; exit 1; }
tail -8 $O/slow_cu.txt

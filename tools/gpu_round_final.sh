#!/bin/bash
# A round's final tree: the whole GPU suite, smoke, the driver's bench command
# (TAG=r03z for round 3: profiles/r03z_*).
set -o pipefail
O=gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'], d['zipf']['value'], d['check_vs_oracle'], d['roofline']['frac'], d['valu_roofline']['frac'], 'e2e', d.get('e2e'))"

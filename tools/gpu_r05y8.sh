#!/bin/bash
# Round 5 final tree (one job corpus across ranks): the whole GPU suite, smoke, the driver's bench command,
# 8-file shares (auto K3 period 4 and P1), then the rocprof evidence
# (kernel-trace window + PMC passes) -> prof_r05y.
set -o pipefail
O=gpurun_out/r05y8
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print('bench20', d['value'], d['fill_drain_gibs'], d['zipf']['value'], d['check_vs_oracle'], d['zipf']['check_vs_oracle'], d['roofline']['frac'], 'e2e', d.get('e2e',{}).get('value'), d['cpu_baseline']['value'], d.get('lifetime'))"
for n in f8_auto f8_p1; do
  a=""; [ $n = f8_p1 ] && a="--k3-period 1"
  timeout -k 10 300 python bench.py --gpus 1 --steps 400 --warmup 8 --files 8 --e2e-steps 0 --no-cpu-baseline --workload random $a > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['fill_drain_gibs'], d['check_vs_oracle'], d['config']['k3_period'], d['kernel_ms_per_step'])"
done
timeout -k 10 1500 tools/profile_round.sh r05y8 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -25 $O/profile.log

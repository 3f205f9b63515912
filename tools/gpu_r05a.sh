#!/bin/bash
# Round 5, first box: the K3 producer-wave microbenchmark (tools/ubench/k3_prod)
# and the round-4 tree's bench line under the driver's command (baseline).
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 180 tools/ubench/k3_prod 64 32768 4096 3 > $O/k3_prod.txt 2>&1; rc=$?
cat $O/k3_prod.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'], d['zipf']['value'], d['check_vs_oracle'], d['roofline']['frac'], d['kernel_ms_per_step'])"

#!/bin/bash
# Round 5: the driver's N = 8 share on one GPU with every leg (random, Zipf, lifetime, e2e, cpu baseline):
# bench.py --files 8 --steps 20 --warmup 5, and 16 files.
set -o pipefail
O=gpurun_out/r05ao
mkdir -p $O
for f in 8 16; do
  timeout -k 10 400 python bench.py --gpus 1 --files $f --steps 20 --warmup 5 > $O/f$f.json 2> $O/f$f.err || { tail -20 $O/f$f.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/f$f.json'));c=d['config']
print('$f files', d['value'], d['fill_drain_gibs'], 'check', d['check_vs_oracle'], 'zipf', d['zipf']['value'], d['zipf']['check_vs_oracle'], 'e2e', d['e2e']['value'], d['e2e']['check_vs_oracle'], 'P', c['k3_period'], 'lag', c['join_lag'], 'life', d.get('lifetime',{}).get('launch_overhead'))"
done

#!/bin/bash
# Residency sweep: the bench with R distinct resident batches (the slice follows
# R), alternating so drift shows.  usage: DEPTHS="32 33 34" tools/gpu_ab_depth.sh
set -o pipefail
O=gpurun_out/depth
mkdir -p $O
python3 -c "import torch;f,t=torch.cuda.mem_get_info();print('free GiB',f/2**30,'total GiB',t/2**30)"
for rep in 1 2; do
  for r in $DEPTHS; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-check --workload random --arenas $r --hbm-frac 0.999 $BENCH_ARGS $EXTRA > $O/d$r.$rep.json 2> $O/d$r.$rep.err || { tail -5 $O/d$r.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/d$r.$rep.json'));print($r, d['value'], d['ms_per_step'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'], d['k3_lanes']['active_chains_mean'])"
  done
done

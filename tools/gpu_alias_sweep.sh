#!/bin/bash
# Residency ceiling: the VALU latency microbenchmark, then the bench with D
# batches in flight over the physical arenas (--alias-depth, read-only inputs
# aliased: the residency a paged arena would free), D = 33 (no aliasing) .. 66.
set -o pipefail
O=gpurun_out/${TAG:-alias}
mkdir -p $O
timeout -k 10 60 tools/ubench/valu_latency > $O/valu_latency.txt 2>&1 || { cat $O/valu_latency.txt; exit 1; }
cat $O/valu_latency.txt
for D in ${DEPTHS:-0 40 48 56 66}; do
  timeout -k 10 240 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check \
      --hbm-frac 0.85 --alias-depth $D > $O/alias_$D.json 2> $O/alias_$D.err || { tail -20 $O/alias_$D.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$O/alias_$D.json'));print($D, d['value'], d['ms_per_step'], d['config']['pipeline_depth'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'], d['k3_lanes'])"
done

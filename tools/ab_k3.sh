#!/bin/bash
# A/B of K3 variant builds on the deep pipeline (auto slice) and alone.
set -o pipefail
O=gpurun_out
for v in base r10 r12 t512 dense; do
  if [ $v = base ]; then L=$PWD/hashbox_amd/libhbxgpu.so; else L=$PWD/build/variants/$v/libhbxgpu.so; fi
  HBX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v', d['value'], d['roofline']['avg_launch_ms'], d['single_batch']['ms'])"
done

#!/bin/bash
# A/B of variant builds on one GPU box, alternating so clock/power drift shows.
# Each variant is a library built under build/variants/<name>/libhbxgpu.so; it
# is copied over the in-tree library for its run (the product loader takes
# only hashbox_amd/libhbxgpu.so), and the in-tree build is restored at the end.
# usage: VARIANTS="a b" BENCH_ARGS="--steps 60" tools/gpu_ab.sh
set -o pipefail
O=gpurun_out
mkdir -p $O build/variants/base
LIB=hashbox_amd/libhbxgpu.so
cp $LIB build/variants/base/libhbxgpu.so
restore() { cp build/variants/base/libhbxgpu.so $LIB; }
trap restore EXIT
for v in base ${VARIANTS} base ${VARIANTS}; do
  cp build/variants/$v/libhbxgpu.so $LIB
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-check $BENCH_ARGS > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done

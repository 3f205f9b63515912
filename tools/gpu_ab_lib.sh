#!/bin/bash
# Parity suite on the in-tree build, then the default bench against variant
# builds (HBX_LIB), alternating so drift shows.  usage: VARIANTS="a b" tools/gpu_ab_lib.sh
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in base ${VARIANTS} base ${VARIANTS}; do
  if [ $v = base ]; then L=$PWD/hashbox_amd/libhbxgpu.so; else L=$PWD/build/variants/$v/libhbxgpu.so; fi
  HBX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done

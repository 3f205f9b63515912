#!/bin/bash
set -o pipefail
O=gpurun_out
HBX_LIB=$PWD/build/variants/dense/libhbxgpu.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "pipelined or edge" > $O/pytest_dense.log 2>&1 || { tail -30 $O/pytest_dense.log; exit 1; }
tail -1 $O/pytest_dense.log
for v in spread:base:0 spread1:base:1 dense:dense:0 dense1:dense:1; do
  IFS=: read tag lib one <<< "$v"
  if [ $lib = base ]; then L=$PWD/hashbox_amd/libhbxgpu.so; else L=$PWD/build/variants/$lib/libhbxgpu.so; fi
  HBX_ONE_STREAM=$one HBX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > $O/ab_$tag.json 2> $O/ab_$tag.err || { tail -5 $O/ab_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$tag.json'));print('$tag', d['value'], d['roofline']['avg_launch_ms'], d['single_batch']['ms'], d['kernel_ms_per_step'])"
done

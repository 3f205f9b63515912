#!/bin/bash
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in base nocoop; do
  if [ $v = base ]; then L=$PWD/hashbox_amd/libhbxgpu.so; else L=$PWD/build/variants/$v/libhbxgpu.so; fi
  HBX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --check > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$v.json'));print('$v', d['value'], d['roofline']['avg_launch_ms'], d['single_batch']['ms'], d['kernel_ms_per_step'], d.get('check_vs_oracle'))"
done
for sl in 16384 8192; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --md5-slice $sl > $O/ab_s$sl.json 2> $O/ab_s$sl.err || { tail -5 $O/ab_s$sl.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_s$sl.json'));print('slice $sl', d['value'], d['roofline']['avg_launch_ms'], d['config']['pipeline_depth'])"
done

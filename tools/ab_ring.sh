#!/bin/bash
# A/B the MD5 prefetch ring depth (variant builds in build/variants/rN)
for r in 4 8 12; do
  HBX_LIB=$PWD/build/variants/r$r/libhbxgpu.so timeout -k 5 100 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --check > gpurun_out/ring_$r.json 2>gpurun_out/ring_err_$r.log || exit 1
  echo ring=$r $(python3 -c "import json;d=json.load(open('gpurun_out/ring_$r.json'));print(d['stages_ms'], d['check_vs_oracle'])")
  HBX_LIB=$PWD/build/variants/r$r/libhbxgpu.so timeout -k 5 200 python tools/validate_config4.py --gib 16 --files 128 > gpurun_out/c4_ring_$r.json 2>gpurun_out/ring_err_$r.log || exit 1
  echo "  config4(16G) $(python3 -c "import json;d=json.load(open('gpurun_out/c4_ring_$r.json'));print(d['gpu_stage_ms'], d['bit_exact'])")"
done

#!/bin/bash
# K3 cooperative stages through LDS-DMA (HBX_K3_DMA, variant builds under
# build/variants/dma<SB><D>): parity of the full-size schedule for the first
# variant, the bench's oracle check for every variant, then alternating A/B
# against the register-staged default.
set -o pipefail
O=gpurun_out/${TAG:-k3dma}
mkdir -p $O build/variants/base
LIB=hashbox_amd/libhbxgpu.so
cp $LIB build/variants/base/libhbxgpu.so
restore() { cp build/variants/base/libhbxgpu.so $LIB; }
trap restore EXIT
V=${VARIANTS:-dma24 dma42 dma18 dma25}
first=${V%% *}
cp build/variants/$first/libhbxgpu.so $LIB
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$first.log 2>&1 || { tail -30 $O/pytest_$first.log; exit 1; }
tail -2 $O/pytest_$first.log
for v in $V; do
  cp build/variants/$v/libhbxgpu.so $LIB
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/check_$v.json 2> $O/check_$v.err || { tail -5 $O/check_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/check_$v.json'));print('$v check', d['check_vs_oracle'], d['value'], d['kernel_ms_per_step'])"
  python3 -c "import json,sys;d=json.load(open('$O/check_$v.json'));sys.exit(0 if d['check_vs_oracle'] is True else 1)" || exit 1
done
restore
VARIANTS="$V" BENCH_ARGS="--steps 100 --workload random" bash tools/gpu_ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt

#!/bin/bash
# State check of the current build on one box: parity suite, the default bench
# line (with the CPU baseline), then A/B of K1 mode 2 (K1-lite, co-resides with
# K3) and a deeper pipeline.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
O=gpurun_out
mkdir -p $O
summ() { python3 -c "import json,sys;d=json.load(open('$1'));print('$2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'], d['config']['pipeline_depth'], d['config']['md5_slice_blocks'], d.get('check_vs_oracle'))"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 60 ./tools/ubench/valu_latency > $O/valu_latency.txt 2>&1 || { cat $O/valu_latency.txt; exit 1; }
cat $O/valu_latency.txt
timeout -k 10 300 python bench.py --check > $O/b_default.json 2> $O/b_default.err || { tail -5 $O/b_default.err; exit 1; }
summ $O/b_default.json default
HBX_K1_MODE=2 timeout -k 10 300 python bench.py --no-cpu-baseline --check > $O/b_k1lite.json 2> $O/b_k1lite.err || { tail -5 $O/b_k1lite.err; exit 1; }
summ $O/b_k1lite.json k1lite
timeout -k 10 300 python bench.py --no-cpu-baseline --hbm-frac 0.9 > $O/b_frac90.json 2> $O/b_frac90.err || { tail -5 $O/b_frac90.err; exit 1; }
summ $O/b_frac90.json frac90

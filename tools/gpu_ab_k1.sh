#!/bin/bash
# Reserved pipeline: parity, bench with K1 mode 1 (LDS-DMA) and 2 (K1-lite),
# then one kernel trace of each for the hash-stream timeline.
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys;d=json.load(open('$1'));print('$2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'], d['config']['pipeline_depth'], d['config']['md5_slice_blocks'], d.get('check_vs_oracle'))"; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for m in ${MODES:-1 2}; do
  HBX_K1_MODE=$m timeout -k 10 300 python bench.py --no-cpu-baseline --check $BENCH_ARGS > $O/ab_k1m$m.json 2> $O/ab_k1m$m.err || { tail -5 $O/ab_k1m$m.err; exit 1; }
  summ $O/ab_k1m$m.json k1mode$m
done
for m in ${MODES:-1 2}; do
  HBX_K1_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl$m -o run -- python3 bench.py --no-cpu-baseline $BENCH_ARGS > $O/tl$m.log 2>&1 || { tail -5 $O/tl$m.log; exit 1; }
  f=$(find $O/tl$m -name "*kernel_trace.csv" | head -1)
  echo "== timeline K1 mode $m"; python3 tools/trace_timeline.py $f 101
done

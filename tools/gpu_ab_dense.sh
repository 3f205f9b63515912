#!/bin/bash
# A/B of K1 kernel (1 LDS-DMA, 2 K1-lite) x K3 placement (0 spread, 1 dense):
# bench line + hash-stream timeline from a kernel trace of the same run.
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in ${CFGS:-1:0 1:1 2:0 2:1}; do
  m=${cfg%%:*}; d=${cfg##*:}; t=m${m}d${d}
  rm -rf $O/tl_$t
  HBX_K1_MODE=$m HBX_K3_DENSE=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$t -o run -- python3 bench.py --no-cpu-baseline $BENCH_ARGS > $O/tl_$t.log 2>&1 || { tail -5 $O/tl_$t.log; exit 1; }
  grep '^{' $O/tl_$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('== $t', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
  f=$(find $O/tl_$t -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_timeline.py $f 101
done

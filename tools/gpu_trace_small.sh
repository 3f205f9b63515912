#!/bin/bash
# Kernel trace of a small-batch pipeline (diagnostics): a few steps of every
# stream in start order, plus the window timeline.
# usage: bash tools/gpu_trace_small.sh <files> <join_lag> [extra bench args]
set -o pipefail
export TMPDIR=/tmp
nf=$1; lag=$2; shift 2
OUT=gpurun_out/trs_${nf}_${lag}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --files $nf --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check --join-lag $lag "$@" > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
KT=$(find $OUT -name "*kernel_trace.csv" | head -1)
grep '^{' $OUT/log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
python3 tools/trace_steps.py $KT -30 3
python3 tools/window_timeline.py $KT 100 | head -4

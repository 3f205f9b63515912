#!/bin/bash
# r01g evidence: default bench (with the CPU baseline and --check), then the rocprof set
set -o pipefail
O=gpurun_out
timeout -k 10 300 python bench.py --check > $O/r01g_bench_default.json 2> $O/r01g_bench.err || { tail -5 $O/r01g_bench.err; exit 1; }
cat $O/r01g_bench_default.json
bash tools/profile_round.sh r01g

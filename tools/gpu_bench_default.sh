#!/bin/bash
set -o pipefail
O=gpurun_out
timeout -k 10 400 python bench.py --check > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json

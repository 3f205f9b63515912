#!/bin/bash
# ${TAG:-r01g} evidence: default bench (with the CPU baseline and --check), then the rocprof set
set -o pipefail
O=gpurun_out
timeout -k 10 300 python bench.py --check > $O/${TAG:-r01g}_bench_default.json 2> $O/${TAG:-r01g}_bench.err || { tail -5 $O/${TAG:-r01g}_bench.err; exit 1; }
cat $O/${TAG:-r01g}_bench_default.json
bash tools/profile_round.sh ${TAG:-r01g}

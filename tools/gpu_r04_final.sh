#!/bin/bash
# Round 4's final tree: the whole GPU suite, smoke, the driver's bench command,
# the rocprof evidence (tools/profile_round.sh: kernel-trace stats of the timed
# window, FETCH_SIZE traffic, SQ and clock counters), then the BASELINE configs
# (1, 3/4, 5) and the deflate/inflate bench.
# usage: TAG=r04z bash tools/gpu_r04_final.sh
set -o pipefail
export TAG=${TAG:-r04z}
bash tools/gpu_round_final.sh || exit 1
bash tools/profile_round.sh $TAG || exit 1
bash tools/gpu_configs.sh || exit 1
timeout -k 10 400 python tools/bench_deflate.py > gpurun_out/deflate_$TAG.json 2> gpurun_out/deflate_$TAG.err || { tail -5 gpurun_out/deflate_$TAG.err; exit 1; }
echo done

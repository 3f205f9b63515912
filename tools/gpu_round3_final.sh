#!/bin/bash
# Round 3's final tree: the whole GPU suite, smoke, the driver's bench command,
# then the rocprof evidence (kernel-trace stats of the timed window, FETCH_SIZE
# traffic, SQ and clock counters) under gpurun_out/prof_$TAG.
# usage: TAG=r03g tools/gpu_round3_final.sh   (default r03f)
set -o pipefail
export TAG=${TAG:-r03f}
bash tools/gpu_round_final.sh || exit 1
bash tools/profile_round.sh $TAG || exit 1

#!/bin/bash
# Round 3's final tree: the whole GPU suite, smoke, the driver's bench command,
# then the rocprof evidence (kernel-trace stats of the timed window, FETCH_SIZE
# traffic, SQ and clock counters) under gpurun_out/prof_r03f.
set -o pipefail
TAG=r03f bash tools/gpu_round_final.sh || exit 1
bash tools/profile_round.sh r03f || exit 1

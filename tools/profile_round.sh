#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the
# repo root): kernel-trace stats of the bench command, then one PMC pass per
# counter group (never combined with other trace domains).
# usage: tools/profile_round.sh <tag> [bench args...]
set -e
TAG=${1:-r01}; shift || true
ARGS=${@:---steps 5 --warmup 1 --no-cpu-baseline}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_l2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_l2.log 2>&1
echo done

#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the
# repo root): kernel-trace stats of the default bench, then PMC passes (one
# counter group each, never combined with other trace domains): HBM traffic
# (FETCH_SIZE) -> profiles/<tag>_traffic.json, and SQ stall/issue counters.
# usage: tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 100 --warmup 10 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 100 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline > $OUT/pmc_sq.log 2>&1 || { tail -5 $OUT/pmc_sq.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum --output-format csv -d $OUT/pmc_tlb -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline > $OUT/pmc_tlb.log 2>&1 || { tail -5 $OUT/pmc_tlb.log; exit 1; }
grep -h "" $OUT/trace.log | tail -1
echo done

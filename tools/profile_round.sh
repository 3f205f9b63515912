#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the
# repo root): kernel-trace stats of the default bench, then PMC passes (one
# counter group each, never combined with other trace domains): HBM traffic
# (FETCH_SIZE) -> <tag>_traffic.json, SQ issue/wait counters, clock.
# usage: tools/profile_round.sh <tag>     (outputs under gpurun_out/prof_<tag>)
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BARGS="--steps 200 --warmup 5 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BARGS > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
grep '^{' $OUT/trace.log > $OUT/bench_under_trace.json
KT=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
KS=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp $KS $OUT/kernel_stats.csv
python3 tools/trace_timed.py $KT $OUT/bench_under_trace.json > $OUT/timed_stats.txt
LAG=$(python3 -c "import json;print(json.load(open('$OUT/bench_under_trace.json'))['config']['join_lag'])")
python3 tools/window_timeline.py $KT 200 --seg=0:20 --seg=20:100 --seg=100:200 --lag=$LAG >> $OUT/timed_stats.txt
cat $OUT/timed_stats.txt
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "hbx_" --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 100 --warmup 2 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $OUT/pmc_fetch.log 2>&1 || { tail -5 $OUT/pmc_fetch.log; exit 1; }
python3 tools/pmc_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $OUT/${TAG}_traffic.json > /dev/null
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --steps 100 --warmup 2 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $OUT/pmc_sq.log 2>&1 || { tail -5 $OUT/pmc_sq.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $OUT/pmc_clk -o run -- python3 bench.py --steps 100 --warmup 2 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $OUT/pmc_clk.log 2>&1 || { tail -5 $OUT/pmc_clk.log; exit 1; }
python3 tools/pmc_k3_summary.py $OUT > $OUT/pmc_summary.txt 2>&1
cat $OUT/${TAG}_traffic.json | python3 -c "import json,sys;d=json.load(sys.stdin);[print(k, v['hbm_bytes']/1e9, 'GB/launch') for k,v in d['kernels'].items()]"
echo done

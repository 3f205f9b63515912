#!/bin/bash
# MD5 issue rate with one and two chains per lane, and the dual-issue counters
# (SQ_ACTIVE_INST_VALU2) of the ubench kernels and of K1/K3 in the bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
timeout -k 10 120 ./tools/ubench/valu_issue x md5 > $O/valu_md5.txt 2>&1 || { cat $O/valu_md5.txt; exit 1; }
cat $O/valu_md5.txt
CTR="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc_ub -o run -- ./tools/ubench/valu_issue x md5_real > $O/pmc_ub.log 2>&1 || { tail -5 $O/pmc_ub.log; exit 1; }
python3 tools/pmc_summary.py --all $O/pmc_ub > $O/pmc_ub_summary.txt; cat $O/pmc_ub_summary.txt
timeout -s KILL 300 rocprofv3 --pmc $CTR --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/pmc_bench -o run -- python3 bench.py --steps 30 --warmup 2 --workload random --no-cpu-baseline --no-check > $O/pmc_bench.log 2>&1 || { tail -5 $O/pmc_bench.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_bench > $O/pmc_bench_summary.txt; cat $O/pmc_bench_summary.txt

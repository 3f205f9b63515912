#!/bin/bash
# VALU issue classes on gfx950 (tools/ubench/valu_issue.hip, every wave
# stamped): stream ops, register-read (distinct operand) ops and MD5 step
# orderings, each with the dual-issue counter SQ_ACTIVE_INST_VALU2; then the
# same counters on K1/K3 inside the bench.  Outputs: profiles/r03c, r03d.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-valu}
mkdir -p $O
CTR="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for sel in v_ distinct md5; do
  timeout -k 10 120 ./tools/ubench/valu_issue x $sel > $O/valu_$sel.txt 2>&1 || { cat $O/valu_$sel.txt; exit 1; }
  cat $O/valu_$sel.txt
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc_$sel -o run -- ./tools/ubench/valu_issue x $sel > $O/pmc_$sel.log 2>&1 || { tail -5 $O/pmc_$sel.log; exit 1; }
  python3 tools/pmc_summary.py --all $O/pmc_$sel > $O/pmc_${sel}_summary.txt
  grep VALU2 $O/pmc_${sel}_summary.txt | head -60
done
timeout -s KILL 300 rocprofv3 --pmc $CTR --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/pmc_bench -o run -- python3 bench.py --steps 30 --warmup 2 --workload random --no-cpu-baseline --no-check > $O/pmc_bench.log 2>&1 || { tail -5 $O/pmc_bench.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_bench > $O/pmc_bench_summary.txt
cat $O/pmc_bench_summary.txt

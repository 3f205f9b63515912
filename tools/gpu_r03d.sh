#!/bin/bash
# Register-read test of the VALU issue classes, with the dual-issue counter.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
timeout -k 10 120 ./tools/ubench/valu_issue x distinct > $O/valu_distinct.txt 2>&1 || { cat $O/valu_distinct.txt; exit 1; }
cat $O/valu_distinct.txt
CTR="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc_d -o run -- ./tools/ubench/valu_issue x distinct > $O/pmc_d.log 2>&1 || { tail -5 $O/pmc_d.log; exit 1; }
python3 tools/pmc_summary.py --all $O/pmc_d > $O/pmc_d_summary.txt
timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $O/pmc_s -o run -- ./tools/ubench/valu_issue x v_ > $O/pmc_s.log 2>&1 || { tail -5 $O/pmc_s.log; exit 1; }
python3 tools/pmc_summary.py --all $O/pmc_s > $O/pmc_s_summary.txt
grep VALU2 $O/pmc_d_summary.txt $O/pmc_s_summary.txt | head -80

#!/bin/bash
# Round 5: host side of the scan loop's long gaps at 8 files per GPU (kernel + HIP runtime trace, no counters).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trace -o run -- python3 bench.py --files 8 --steps 100 --warmup 8 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
ls $O/trace/*/ 2>/dev/null | head; find $O/trace -name "*.csv" | head
python3 tools/host_gaps.py $O/trace 100 3 > $O/host_gaps.txt 2>&1
head -80 $O/host_gaps.txt

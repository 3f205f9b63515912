#!/bin/bash
# Round 5: where the scan loop's gaps go at 8 files per GPU with K3 period 4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05k}
mkdir -p $O
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --files 8 --k3-period 4 --steps 200 --warmup 8 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime $BEXTRA > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
KT=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 tools/scan_gaps.py $KT 150 --show 6 > $O/scan_gaps.txt
cat $O/scan_gaps.txt | head -80
grep '^{' $O/trace.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['kernel_ms_per_step'])"

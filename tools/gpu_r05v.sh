#!/bin/bash
# Round 5: what a 20-step window (the driver's command) holds: kernel trace of bench.py --steps 20 --warmup 5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
for k in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace$k -o run -- python3 bench.py --steps 20 --warmup 5 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $O/trace$k.log 2>&1 || { tail -5 $O/trace$k.log; exit 1; }
KT=$(find $O/trace$k -name "*kernel_trace.csv" | head -1)
grep '^{' $O/trace$k.log > $O/bench$k.json
python3 -c "import json;d=json.load(open('$O/bench$k.json'));print('bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['host_ms_per_step'])"
python3 tools/window_timeline.py $KT 20 --all --lag=2 > $O/timeline$k.txt 2>&1
cat $O/timeline$k.txt | tail -30
done

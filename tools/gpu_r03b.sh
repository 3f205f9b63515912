#!/bin/bash
# VALU issue classes (every wave stamped) and the driver's bench command.
set -o pipefail
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
timeout -k 10 200 ./tools/ubench/valu_issue > $O/valu_issue.txt 2>&1 || { cat $O/valu_issue.txt; exit 1; }
cat $O/valu_issue.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
cat $O/bench20.json

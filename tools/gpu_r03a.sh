#!/bin/bash
# Round-3 first pass: the whole GPU parity suite on the round-2 head, smoke, and
# the aggregate VALU issue-rate microbenchmark (every wave stamped).
set -o pipefail
O=gpurun_out/${TAG:-r03a}
mkdir -p $O
timeout -k 10 120 ./tools/ubench/valu_issue > $O/valu_issue.txt 2>&1 || { cat $O/valu_issue.txt; exit 1; }
cat $O/valu_issue.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log

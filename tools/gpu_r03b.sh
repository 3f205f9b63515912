#!/bin/bash
# VALU issue classes (every wave stamped), the available SQ counters, the new
# config parity tests, smoke with a pipelined batch, the driver's bench.
set -o pipefail
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
timeout -k 10 200 ./tools/ubench/valu_issue > $O/valu_issue.txt 2>&1 || { cat $O/valu_issue.txt; exit 1; }
cat $O/valu_issue.txt | tail -50
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/$O/counters.txt 2>&1) || echo "counter list failed"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_abi.py -x -v --timeout 400 --timeout-method thread > $O/pytest_cfg.log 2>&1 || { tail -40 $O/pytest_cfg.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_cfg.log | tail -20
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
cat $O/bench20.json

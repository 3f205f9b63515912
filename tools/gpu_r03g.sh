#!/bin/bash
# K3 LDS prefetch: parity, then A/B against no prefetch and against compiler H rounds.
set -o pipefail
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
VARIANTS="nopf noxad" BENCH_ARGS="--steps 100 --workload random" bash tools/gpu_ab.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt

#!/bin/bash
# Round-2 first pass: GPU parity suite, smoke, the driver's bench command and a
# long steady-state bench (the two headlines must agree within a few %).
set -o pipefail
O=gpurun_out/${TAG:-r02a}
mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>&1; python3 -c "import os;print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 300 python bench.py --steps 600 --warmup 5 --workload random --no-cpu-baseline > $O/bench600.json 2> $O/bench600.err || { tail -20 $O/bench600.err; exit 1; }
cat $O/bench600.json

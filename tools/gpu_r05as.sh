#!/bin/bash
# Round 5: is the one slow submit of a 20-step window at 8 files a CPU-quota throttle of the box's cgroup?
set -o pipefail
O=gpurun_out/r05as
mkdir -p $O
{ cat /proc/self/cgroup; for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us; do echo "== $f"; cat $f 2>&1; done; nproc; } > $O/cgroup.txt 2>&1
cat $O/cgroup.txt
run() {
  local n=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 --files 8 --e2e-steps 0 --no-cpu-baseline --no-lifetime --no-check --workload random "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d['host_ms_per_step'])"
}
run w5 --steps 20 --warmup 5 || exit 1
run w5b --steps 20 --warmup 5 || exit 1
OMP_NUM_THREADS=4 run w5omp4 --steps 20 --warmup 5 || exit 1

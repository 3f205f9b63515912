#!/bin/bash
# Config 5 host reads: the engine's CPU use and cgroup throttling during
# store_paths, then the C++ read microbenchmark on the very same files.
set -o pipefail
O=gpurun_out/c5diag; mkdir -p $O
timeout -k 10 300 python tools/bench_config5.py --cpu-sample 200 --keep --io-threads ${IO:-16} > $O/c5.json 2> $O/c5.err || { tail -3 $O/c5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1])
print(d['e2e_gibs'], d['passes'], d['sample_mismatches'])"
RD_DIR=/dev/shm/hbx_config5 RD_BATCH=1700 timeout -k 10 200 tools/ubench/read_files > $O/ub.txt 2>&1; rc=$?
cat $O/ub.txt
rm -rf /dev/shm/hbx_config5
exit $rc

#!/bin/bash
# Config 5 host-read scaling: io threads and batch size (files made once, kept between runs).
set -o pipefail
O=gpurun_out/c5io; mkdir -p $O
first=1
for cfg in ${CFGS:-"16 1024" "12 1024" "14 1024" "10 1024"}; do
  set -- $cfg
  keep="--keep"
  timeout -k 10 300 python tools/bench_config5.py --io-threads $1 --batch-mib $2 --cpu-sample 200 $keep > $O/c5_$1_$2.json 2> $O/c5.err || { tail -3 $O/c5.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c5_$1_$2.json').read().strip().splitlines()[-1])
print('io=$1 batch=$2', d['e2e_gibs'], d['host_seconds'], d['sample_mismatches'])"
done
rm -rf /dev/shm/hbx_config5

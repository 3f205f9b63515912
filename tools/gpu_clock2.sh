#!/bin/bash
# GFX clock and power in steady state: the default pipeline (K1 beside K3) vs
# the serialized schedule (HBX_HASH_CUS=0:4096: K3 never overlaps K1), with
# rocm-smi sampling beside each long bench.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/clock2
mkdir -p $O
one() {  # name, HBX_HASH_CUS
  (HBX_HASH_CUS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4000 > $O/$1.json 2> $O/$1.err; echo "bench rc=$?" >> $O/$1.err) &
  BP=$!
  sleep 12
  for i in $(seq 1 40); do
    kill -0 $BP 2>/dev/null || break
    timeout 10 rocm-smi --showclocks --showpower >> $O/$1_smi.log 2>&1
    sleep 0.3
  done
  wait $BP
  tail -1 $O/$1.err
  python3 -c "import json;d=json.load(open('$O/$1.json'));print('$1', d['value'], d['kernel_ms_per_step'])"
  grep -E "sclk|Power" $O/$1_smi.log | sort | uniq -c | sort -rn | head -12
}
one pipelined ""
one serialized 0:4096

#!/bin/bash
# A/B: K1 (scan stream) and K3 (hash stream) on disjoint CU sets via stream CU masks
set -o pipefail
O=gpurun_out
run() {  # name, HBX_HASH_CUS, HBX_SCAN_CUS
  HBX_HASH_CUS=$2 HBX_SCAN_CUS=$3 timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/cm_$1.json 2> $O/cm_$1.err || { tail -5 $O/cm_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cm_$1.json'));print('$1', '$2', '$3', d['value'], d['kernel_ms_per_step'], d.get('check_vs_oracle'))"
}
run base "" ""
run h128s128 0:128 128:128
run h128s128i 0:128:2 1:128:2
run h144s112 0:144 144:112
run h160all 0:160 ""
run h144i_sall 0:144:1 0:256
run base2 "" ""

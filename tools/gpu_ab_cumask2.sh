#!/bin/bash
# A/B: does a CU-masked stream by itself serialize K1 and K3?
set -o pipefail
O=gpurun_out
run() {  # name, HBX_HASH_CUS, HBX_SCAN_CUS
  HBX_HASH_CUS=$2 HBX_SCAN_CUS=$3 timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cm_$1.json 2> $O/cm_$1.err || { tail -5 $O/cm_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cm_$1.json'));print('$1', '$2', '$3', d['value'], d['kernel_ms_per_step'])"
}
run hfull_sfull 0:256 0:256
run hnone_sfull "" 0:256
run hfull_snone 0:256 ""
run hnone_si "" 1:128:2
run hnone_s192 "" 64:192

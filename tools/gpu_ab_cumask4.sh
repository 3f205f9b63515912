#!/bin/bash
# A/B: K1 intensity through the scan stream's CU set (the hash stream stays unmasked)
set -o pipefail
O=gpurun_out
run() {  # name, HBX_SCAN_CUS
  HBX_SCAN_CUS=$2 timeout -k 10 180 python bench.py --no-cpu-baseline > $O/cm4_$1.json 2> $O/cm4_$1.err || { tail -5 $O/cm4_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cm4_$1.json'));print('$1', '$2', d['value'], d['kernel_ms_per_step'])"
}
run full 0:4096
run c240 16:240
run c224 32:224
run c208 48:208
run full2 0:4096
run c224b 32:224
run c240b 16:240

#!/bin/bash
# A/B: scan stream (and result stream) created through the CU-mask API with a full mask
set -o pipefail
O=gpurun_out
run() {  # name, HBX_SCAN_CUS, HBX_RES_CUS
  HBX_SCAN_CUS=$2 HBX_RES_CUS=$3 timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/cm3_$1.json 2> $O/cm3_$1.err || { tail -5 $O/cm3_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cm3_$1.json'));print('$1', '$2', '$3', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
}
run base "" ""
run sfull 0:256 ""
run base2 "" ""
run sfull2 0:256 ""
run sfull_rfull 0:256 0:256
run rfull "" 0:256
run sfull3 0:256 ""

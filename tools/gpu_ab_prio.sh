#!/bin/bash
# A/B: stream priorities for the hash stream (K3) and the scan stream (K1/K2)
set -o pipefail
O=gpurun_out
run() {  # name, HBX_HASH_CUS, HBX_SCAN_CUS
  HBX_HASH_CUS=$2 HBX_SCAN_CUS=$3 timeout -k 10 180 python bench.py --no-cpu-baseline --check > $O/pr_$1.json 2> $O/pr_$1.err || { tail -5 $O/pr_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/pr_$1.json'));print('$1', '$2', '$3', d['value'], d['kernel_ms_per_step'], d['check_vs_oracle'])"
}
run base off 0:4096
run hhi prio:hi 0:4096
run hhi_soff prio:hi off
run hoff_slo off prio:lo
run hhi_slo prio:hi prio:lo
run hlo prio:lo 0:4096
run base2 off 0:4096

#!/bin/bash
# Round 5: results to the host by a kernel (hbx_result_push) instead of the SDMA copy whose call stalled one
# submit ~7 ms: the 20-step window at 8 files, and the driver's 64-file command, both ways, with the oracle check.
set -o pipefail
O=gpurun_out/r05az
mkdir -p $O
run() {
  local n=$1; shift
  HBX_TRACE_SLOW_SUBMIT=2 timeout -k 10 300 python bench.py --gpus 1 --e2e-steps 0 --no-cpu-baseline --no-lifetime "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  grep -c "slow submit" $O/$n.err
  python3 -c "
import json;d=json.load(open('$O/$n.json'))
print('$n', d['value'], d.get('check_vs_oracle'), d['host_ms_per_step'], 'zipf', d.get('zipf',{}).get('value'))"
}
run f8sdma --files 8 --steps 20 --warmup 5 || exit 1
HBX_AB=1 HBX_D2H_KERNEL=64 run f8k64 --files 8 --steps 20 --warmup 5 || exit 1
HBX_AB=1 HBX_D2H_KERNEL=16 run f8k16 --files 8 --steps 20 --warmup 5 || exit 1
run b64sdma --steps 20 --warmup 5 || exit 1
HBX_AB=1 HBX_D2H_KERNEL=64 run b64k64 --steps 20 --warmup 5 || exit 1

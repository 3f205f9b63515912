#!/bin/bash
# K3 memory-side counters in two regimes: one batch alone (slice 0) and the
# deep pipeline (slice 5699, 24 batches).  One PMC group per pass.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_k3
mkdir -p $O
run() {  # tag, slice, counters...
  local tag=$1 slice=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex hbx_k3 --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --md5-slice $slice > $O/$tag.log 2>&1
}
for cfg in "s0 0" "s5699 5699"; do
  set -- $cfg
  run ${1}_sq $2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES || exit 1
  run ${1}_tlb $2 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum || exit 1
  run ${1}_tcc $2 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE || exit 1
  run ${1}_utcl $2 TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_SERIALIZATION_STALL_sum || exit 1
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

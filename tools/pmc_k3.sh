#!/bin/bash
# K3 counters in the deep pipeline (auto slice), one PMC group per pass;
# tools/pmc_k3_summary.py prints the median over steady-state dispatches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_k3b
mkdir -p $O
run() {  # tag, counters...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES || exit 1
run tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_LATENCY_sum TCP_TA_TCP_STATE_READ_sum || exit 1
run lds SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
python3 tools/pmc_k3_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

#!/bin/bash
# K3 counters in the STEADY state of the default pipeline (100 steps; the
# summary takes the middle third of the dispatches): clock and issue.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_k3d
mkdir -p $O
run() {  # tag, counters...
  local tag=$1; shift
  HBX_K1_MODE=${K1MODE:-2} timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 100 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1
}
run clk GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVES || exit 1
python3 tools/pmc_k3_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

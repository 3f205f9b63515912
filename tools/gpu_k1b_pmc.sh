#!/bin/bash
# K1 vs K1b under PMC (kernels serialized: each runs alone on the chip):
# VALU instructions, wave cycles, issue activity.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k1b_pmc}
mkdir -p $O
for R in 64 128; do
  HBX_K1_RUN=$R timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "hbx_k1" --output-format csv -d $O/pmc_$R -o run -- python3 bench.py --steps 30 --warmup 2 --workload random --no-cpu-baseline --no-check > $O/pmc_$R.log 2>&1 || { tail -5 $O/pmc_$R.log; exit 1; }
  python3 tools/pmc_k3_summary.py $O/pmc_$R > $O/summary_$R.txt 2>&1
  grep -A14 "^hbx_k1_digest" $O/summary_$R.txt
done

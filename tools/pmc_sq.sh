#!/bin/bash
# SQ stall breakdown + clock for the bench kernels (one PMC pass per group).
set -e
TAG=${1:-sq}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/sq -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/grbm -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/grbm.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d $OUT/sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq2.log 2>&1
echo done

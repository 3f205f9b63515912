#!/bin/bash
# K7a (tools/ubench/k7_phases.hip, 256 MiB Zipf text) under rocprofv3: kernel
# stats, then one PMC pass of SQ counters (LDS vs VALU vs waits).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/k7pmc
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ihashbox_amd/csrc -o $O/k7_phases tools/ubench/k7_phases.hip || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- $O/k7_phases 256 > $O/stats.log 2>&1 || { tail -5 $O/stats.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d $O/pmc -o run -- $O/k7_phases 256 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
find $O -name "*.csv" | head

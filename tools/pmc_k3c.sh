#!/bin/bash
# K3 in the deep pipeline: the bench with scan and hash on one stream (K3
# alone on the chip), then counters, one PMC group per pass (kernels are
# serialized under --pmc): issue/wait, clock, instruction cache.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_k3c
mkdir -p $O
HBX_ONE_STREAM=1 HBX_K1_MODE=2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/one_stream.json 2> $O/one_stream.err || { tail -5 $O/one_stream.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/one_stream.json'));print('one stream', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'])"
run() {  # tag, counters...
  local tag=$1; shift
  HBX_K1_MODE=2 timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/$tag -o run -- python3 bench.py --steps 30 --warmup 2 --no-cpu-baseline > $O/$tag.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES || exit 1
run clk GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC || exit 1
run ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES || { tail -5 $O/ic.log; echo "ic pass failed"; }
python3 tools/pmc_k3_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt

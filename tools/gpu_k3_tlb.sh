#!/bin/bash
# K3 address translation: one 2 MiB-aligned allocation for all arenas
# (--single-alloc) vs one allocation per arena; UTCL1 misses per launch and the
# bench value for each.  Output: profiles/r03h.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k3tlb}
mkdir -p $O
for m in default single; do
  F=""; [ $m = single ] && F="--single-alloc"
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check $F > $O/bench_$m.json 2> $O/bench_$m.err || { tail -5 $O/bench_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['kernel_ms_per_step'])"
  timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/pmc_$m -o run -- python3 bench.py --steps 30 --warmup 2 --workload random --no-cpu-baseline --no-check $F > $O/pmc_$m.log 2>&1 || { tail -5 $O/pmc_$m.log; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_$m | grep -v gate
done

#!/bin/bash
# K7 with a 16 KiB history window, 8-way buckets and resolved thread ranges:
# strict-inflate tests, the deflate bench; then K3 address translation: one
# 2 MiB-aligned allocation for all arenas vs one allocation per arena.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_inflate.py tests/test_gpu_wire.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/bench_deflate.py > $O/deflate.json 2> $O/deflate.err || { tail -20 $O/deflate.err; exit 1; }
cat $O/deflate.json
for m in default single; do
  F=""; [ $m = single ] && F="--single-alloc"
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check $F > $O/bench_$m.json 2> $O/bench_$m.err || { tail -5 $O/bench_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$m.json'));print('$m', d['value'], d['kernel_ms_per_step'])"
  timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex "hbx_k3|hbx_k1" --output-format csv -d $O/pmc_$m -o run -- python3 bench.py --steps 30 --warmup 2 --workload random --no-cpu-baseline --no-check $F > $O/pmc_$m.log 2>&1 || { tail -5 $O/pmc_$m.log; exit 1; }
  python3 tools/pmc_summary.py $O/pmc_$m | grep -v gate
done

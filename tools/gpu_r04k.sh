#!/bin/bash
# Round 4, K7 ratio (verdict item 7): K7h, shared dynamic codes over groups of four segments.
# phase probe (text and random), then bench_deflate (ratio, speed, CPU).
set -o pipefail
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_inflate.py -x -v --timeout 300 --timeout-method thread > $O/pytest_deflate.log 2>&1 || { tail -40 $O/pytest_deflate.log; exit 1; }
tail -2 $O/pytest_deflate.log
hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ihashbox_amd/csrc -o $O/k7_phases tools/ubench/k7_phases.hip
timeout -k 10 120 $O/k7_phases 256 > $O/k7_phases.txt 2>&1 && timeout -k 10 120 $O/k7_phases 256 random >> $O/k7_phases.txt 2>&1 || { cat $O/k7_phases.txt; exit 1; }
cat $O/k7_phases.txt
timeout -k 10 400 python tools/bench_deflate.py > $O/deflate.json 2> $O/deflate.err || { tail -5 $O/deflate.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/deflate.json'));print(json.dumps(d)[:3000])"

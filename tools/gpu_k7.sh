#!/bin/bash
# K7 (history window, parallel candidates, repeat-aware early-out): strict
# inflate tests, the deflate bench, phase times.
set -o pipefail
O=gpurun_out/${TAG:-k7}
mkdir -p $O
timeout -k 10 120 ./tools/ubench/k7_phases 256 > $O/k7_phases0.txt 2>&1 || { cat $O/k7_phases0.txt; exit 1; }
cat $O/k7_phases0.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_inflate.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/bench_deflate.py > $O/deflate.json 2> $O/deflate.err || { tail -20 $O/deflate.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/deflate.json'));print({k:(d[k].get('ratio'),d[k].get('gbs')) for k in ('random','text')})"
timeout -k 10 120 ./tools/ubench/k7_phases 256 > $O/k7_phases.txt 2>&1 && timeout -k 10 120 ./tools/ubench/k7_phases 256 random >> $O/k7_phases.txt 2>&1 || { cat $O/k7_phases.txt; exit 1; }
cat $O/k7_phases.txt

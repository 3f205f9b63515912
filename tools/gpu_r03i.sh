#!/bin/bash
# K7 candidate pruning: strict-inflate tests and the deflate bench.
set -o pipefail
O=gpurun_out/${TAG:-r03i}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/bench_deflate.py > $O/deflate.json 2> $O/deflate.err || { tail -20 $O/deflate.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/deflate.json'));print({k:(d[k].get('ratio'),d[k].get('gbs')) for k in ('random','text')})"

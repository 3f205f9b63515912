#!/bin/bash
# Round 4: K8s first (inflate tests in every mode, the deflate/inflate bench),
# then the final tree's suite, smoke and the driver's bench command.  The
# rocprof evidence and the configs follow in tools/gpu_r04e.sh (the 1,200 s
# limit per call).
set -o pipefail
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_deflate.py -x -v --timeout 300 --timeout-method thread > $O/pytest_inflate.log 2>&1 || { tail -40 $O/pytest_inflate.log; exit 1; }
tail -2 $O/pytest_inflate.log
timeout -k 10 400 python tools/bench_deflate.py > $O/deflate.json 2> $O/deflate.err || { tail -5 $O/deflate.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/deflate.json'));print(d['text']['inflate_device'], d['text'].get('inflate_zlib6_device'))"
TAG=r04z bash tools/gpu_round_final.sh

#!/bin/bash
# Asynchronous compression in the disk path: the store_paths / deflate /
# inflate / wire GPU tests, then config 5 with every chunk compressed.
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/${TAG:-zpipe}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "store_paths or tree or deflate or wire or inflate" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 env HBX_ZDIAG=1 python tools/bench_config5.py --compress > $O/config5.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/config5.json').read().strip().splitlines()[-1])
print('config5', d['e2e_gibs'], d['host_seconds'], d['sample_mismatches'])
print('compressed', d['compressed'])"
grep zdiag $O/config5.err

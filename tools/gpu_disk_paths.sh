#!/bin/bash
# The disk paths on the current build: store_paths tests, config 5 (two passes,
# plus compression), the whole-tree store.
set -o pipefail
O=gpurun_out/disk; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "store_paths or tree" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python tools/bench_config5.py --compress > $O/config5.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/config5.json').read().strip().splitlines()[-1])
print('config5', d['e2e_gibs'], d['passes'], d['host_seconds'], d['sample_mismatches'], d['cpu_oracle']['gibs'])
print('compressed', d['compressed'])"
timeout -k 10 400 python tools/bench_tree.py > $O/tree.json 2> $O/tree.err || { tail -5 $O/tree.err; exit 1; }
cat $O/tree.json

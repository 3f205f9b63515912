#!/bin/bash
# parity suite, then the default bench (with --check)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --check > $O/bq.json 2> $O/bq.err || { tail -5 $O/bq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bq.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step'], d['single_batch']['ms'], d.get('check_vs_oracle'))"

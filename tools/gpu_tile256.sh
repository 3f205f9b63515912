#!/bin/bash
# tile_iters 256 default: parity suite, smoke, default bench, the BASELINE configs
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py --check > $O/t256_bench.json 2> $O/t256_bench.err || { tail -5 $O/t256_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/t256_bench.json'));print(d['value'], d['kernel_ms_per_step'], d['single_batch'], d['check_vs_oracle'])"
bash tools/gpu_configs.sh

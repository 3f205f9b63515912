#!/bin/bash
# K1b (128-byte runs, 512 threads): parity, then the bench A/B against K1 at
# the default residency (lead 2) and at lead 1 (hbx_input_after_oldest).
set -o pipefail
export HBX_AB=1  # the library honours HBX_* A/B switches only with this
O=gpurun_out/${TAG:-k1b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_k1b.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "64 -1" "128 -1" "64 1" "128 1" "128 -1"; do
  set -- $cfg
  timeout -k 10 240 env HBX_K1_RUN=$1 python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --lead $2 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -20 $O/bench_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$1_$2.json'));print('run $1 lead $2', d['value'], d['ms_per_step'], d.get('check_vs_oracle'), d['kernel_ms_per_step'], d['config']['md5_slice_blocks'])"
done

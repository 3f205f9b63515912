#!/bin/bash
# K3 with three register sets of cooperative loads (HBX_K3_SETS=3) vs two,
# alternating, at the default residency; one parity test of the variant.
set -o pipefail
O=gpurun_out/${TAG:-k3s3}; mkdir -p $O
HBX_K3_SETS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -k "configs1 and 1" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for S in 2 3; do
  timeout -k 10 240 env HBX_K3_SETS=$S python bench.py --steps 100 --warmup 5 --workload random --no-cpu-baseline --no-check > $O/s${S}_$i.json 2> $O/s${S}_$i.err || { tail -20 $O/s${S}_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/s${S}_$i.json'));print('sets $S run $i', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done; done

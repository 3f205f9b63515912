#!/bin/bash
# K3 tail cut: its parity tests, then bench A/B (alternating) at 8 and 64 files.
set -o pipefail
O=gpurun_out/tailcut
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "tail_cut or pipelined or reserved or input" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for nf in ${NFILES:-8 64}; do
  for rep in 1 2; do
    for v in ${CUTS:-0 90}; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --workload random --steps ${STEPS:-200} --files $nf --e2e-steps 0 --tail-cut $v \
        > $O/b_${nf}_${v}_${rep}.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/b_${nf}_${v}_${rep}.json').read().strip().splitlines()[-1]);print('files',$nf,'cut',$v,'rep',$rep,d['value'],d['kernel_ms_per_step'].get('k3_block_md5'),d['ms_per_step'],d['check_vs_oracle'],d['config']['md5_slice_blocks'],d['config']['launches_per_batch'])"
    done
  done
done

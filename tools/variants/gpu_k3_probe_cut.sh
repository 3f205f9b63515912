#!/bin/bash
# K3 per-wave timeline with and without the tail cut (8 files).
set -o pipefail
for v in 0 97; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-check --workload random --steps 50 --files ${NF:-8} --k3-probe --e2e-steps 0 --tail-cut $v \
    > gpurun_out/probe_cut_$v.json 2> gpurun_out/probe.err || { tail -3 gpurun_out/probe.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/probe_cut_$v.json').read().strip().splitlines()[-1]);p=d['k3_probe'];print($v, d['value'], d['kernel_ms_per_step']['k3_block_md5'], {k:p[k] for k in ('busy_waves','span_us','startup_us_min_med_max','end_us_min_med_max','R_min_med_max','full_slice_waves','full_slice_end_us_min_med_max')})"
done

#!/bin/bash
set -o pipefail
O=gpurun_out
for w in 256 224 192 160 128; do
  HBX_MD5_WGS=$w timeout -k 10 200 python bench.py --no-cpu-baseline > $O/wgs_$w.json 2> $O/wgs_$w.err || { tail -5 $O/wgs_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/wgs_$w.json'));print('wgs $w', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done

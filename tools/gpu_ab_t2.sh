#!/bin/bash
# A/B: K1 tile 256 / 512 / 1024 and the K3 slice length
set -o pipefail
O=gpurun_out
run() {  # name, tile, extra bench args
  HBX_TILE_ITERS=$2 timeout -k 10 180 python bench.py --no-cpu-baseline $3 > $O/t2_$1.json 2> $O/t2_$1.err || { tail -5 $O/t2_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t2_$1.json'));print('$1', d['value'], d['config']['md5_slice_blocks'], d['kernel_ms_per_step'])"
}
run t256 256 ""
run t512 512 ""
run t1024 1024 ""
run t256b 256 ""
run t512b 512 ""
run t1024b 1024 ""
run t256_s3000 256 "--md5-slice 3000"
run t256_s6000 256 "--md5-slice 6000"

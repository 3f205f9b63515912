#!/bin/bash
# Round 4, after pruning the product library: the whole GPU suite, the driver's
# bench command, then K3's memory side at 64 vs 32 chains per wave
# (tools/ubench/hbm_streams, verdict r03 item 4).
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'], d['zipf']['value'], d['check_vs_oracle'], d['roofline']['frac'], 'e2e', d['e2e']['value'], d['e2e']['check_vs_oracle'])"
timeout -k 10 300 tools/ubench/hbm_streams 128 > $O/hbm_streams_cpw.txt 2>&1 || { tail -5 $O/hbm_streams_cpw.txt; exit 1; }
cat $O/hbm_streams_cpw.txt

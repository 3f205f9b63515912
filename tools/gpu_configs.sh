#!/bin/bash
# BASELINE configs 1, 3/4, 5 and the PCIe-inclusive rate on the current build.
set -o pipefail
O=gpurun_out
timeout -k 10 200 python tools/bench_config1.py > $O/config1.json 2> $O/config1.err || { tail -5 $O/config1.err; exit 1; }
cat $O/config1.json
timeout -k 10 400 python tools/validate_config4.py > $O/config4.json 2> $O/config4.err || { tail -5 $O/config4.err; exit 1; }
cat $O/config4.json
timeout -k 10 200 python bench.py --e2e --steps 20 --warmup 3 > $O/e2e.json 2> $O/e2e.err || { tail -5 $O/e2e.err; exit 1; }
cat $O/e2e.json
timeout -k 10 600 python tools/bench_config5.py > $O/config5.json 2> $O/config5.err || { tail -5 $O/config5.err; exit 1; }
cat $O/config5.json

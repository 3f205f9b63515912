#!/bin/bash
# Round 5 final kernels: config 5 end to end (100 k files on tmpfs) and the wire loopback.
set -o pipefail
O=gpurun_out/r05am
mkdir -p $O
timeout -k 10 400 python tools/bench_config5.py --files 100000 > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/config5.json'));print('config5', d['e2e_gibs'], d['sample_mismatches'], d.get('host_seconds'))"
timeout -k 10 400 python tools/bench_wire.py --files 100000 > $O/wire.json 2> $O/wire.err || { tail -20 $O/wire.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/wire.json'));print('wire', d['end_to_end_gibs'], d['store_gibs'], d['sink']['verify_failures'], d['failed'])"

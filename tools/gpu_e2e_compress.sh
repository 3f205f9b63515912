#!/bin/bash
# End-to-end paths with the round-3 K7: config 5 with every chunk compressed,
# and the disk -> zlib -> socket -> sink wire loopback.
set -o pipefail
O=gpurun_out/${TAG:-e2e}
mkdir -p $O
timeout -k 10 500 python tools/bench_config5.py --compress > $O/config5_compressed.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
cat $O/config5_compressed.json
timeout -k 10 600 python tools/bench_wire.py > $O/wire.json 2> $O/wire.err || { tail -20 $O/wire.err; exit 1; }
cat $O/wire.json

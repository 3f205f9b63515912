#!/bin/bash
# Round 5 evidence on the final kernels: rocprofv3 kernel-trace of the bench
# window + PMC passes (FETCH_SIZE traffic, SQ, clock/UTCL1) -> prof_r05z;
# config 5 end to end (100 k files on tmpfs, plain and compressed); the wire
# loopback (hbx_wire_e2e: disk -> zlib -> socket -> re-verifying sink).
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 1500 tools/profile_round.sh r05z > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -25 $O/profile.log
timeout -k 10 400 python tools/bench_config5.py --files 100000 > $O/config5.json 2> $O/config5.err || { tail -20 $O/config5.err; exit 1; }
tail -c 1500 $O/config5.json
timeout -k 10 400 python tools/bench_wire.py --files 100000 > $O/wire.json 2> $O/wire.err || { tail -20 $O/wire.err; exit 1; }
tail -c 1500 $O/wire.json

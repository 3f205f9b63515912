#!/bin/bash
# Round 5: the one slow submit of a 20-step window at 8 files: HIP calls longer than 1 ms (HIP runtime trace).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aq
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-runtime-trace --output-format csv -d $O/trace -o run -- python3 bench.py --files 8 --steps 20 --warmup 5 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
F=$(find $O/trace -name "*hip_api_trace.csv" | head -1)
python3 - "$F" <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(sys.argv[1])))
t0 = rows[0][0]
long = [(s, e, f) for s, e, f in rows if e - s > 1_000_000]
print("calls", len(rows), "longer than 1 ms:", len(long))
for s, e, f in long[-25:]:
    print(f"  {(s - t0) / 1e6:10.2f} ms  {(e - s) / 1e6:8.2f} ms  {f}")
PY
grep '^{' $O/trace.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['host_ms_per_step'])"

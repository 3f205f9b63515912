#!/bin/bash
# SQ counters of the inflate kernel (K8) over tools/bench_deflate.py (one PMC pass).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/k8pmc; mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --kernel-include-regex "hbx_k8" --output-format csv -d $OUT -o run -- python3 tools/bench_deflate.py > $OUT/log 2>&1 || { tail -5 $OUT/log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/k8pmc/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    key = (r["Dispatch_Id"], r["Grid_Size"])
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY

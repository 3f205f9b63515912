#!/bin/bash
# Round 5: where K1's (and K3P's) waves stall: one SQ PMC pass (LDS issue stalls, bank conflicts, active VALU/LDS).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex "hbx_k3p|hbx_k1_digest" --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 60 --warmup 2 --workload random --no-cpu-baseline --no-check --e2e-steps 0 --no-lifetime > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
F=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[k].add(r["Dispatch_Id"])
for k, d in agg.items():
    n = len(cnt[k])
    print(k, "dispatches", n)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v / n:.4g}")
    w = d.get("SQ_WAVE_CYCLES", 0) or 1
    print("   per wave-cycle: wait_any %.3f wait_inst_any %.3f wait_inst_lds %.3f active_valu %.3f active_lds %.3f; bank conflicts / active_lds %.3f" % (
        d.get("SQ_WAIT_ANY", 0) / w, d.get("SQ_WAIT_INST_ANY", 0) / w, d.get("SQ_WAIT_INST_LDS", 0) / w,
        d.get("SQ_ACTIVE_INST_VALU", 0) / w, d.get("SQ_ACTIVE_INST_LDS", 0) / w,
        d.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, d.get("SQ_ACTIVE_INST_LDS", 0))))
PY

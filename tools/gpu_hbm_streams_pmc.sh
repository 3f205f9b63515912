#!/bin/bash
# UTCL1 translation hits/misses of K3's load pattern without the MD5
# (tools/ubench/hbm_streams): chains at random offsets vs a wave's chains in
# one 2 MiB page vs contiguous, 32k chains, one rocprofv3 --pmc pass each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hbms_pmc
mkdir -p $O
for c in coop_lds2_rand coop_lds2_page coop_lds2_local; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex coop --output-format csv -d $O/$c -o run -- ./tools/ubench/hbm_streams 128 $c 32768 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
  tail -1 $O/$c.log
  python3 - "$O/$c" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for row in csv.DictReader(open(f)):
    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
h, mi = m.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0), m.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0)
print("  per dispatch: utcl1 hit %.3g miss %.3g miss-rate %.3f  wait/wave-cycles %.3f" % (h, mi, mi / max(1, h + mi), m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1))))
PY
done

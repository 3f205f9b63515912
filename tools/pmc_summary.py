"""Average rocprofv3 counter values per kernel: python tools/pmc_summary.py [--all] <dir>...
(--all: every kernel, not only the engine's hbx_* kernels)"""
import collections
import csv
import glob
import sys

ALL = "--all" in sys.argv
for d in [x for x in sys.argv[1:] if x != "--all"]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(r["Kernel_Name"][:28], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in sorted(agg.items()):
            if ALL or k.startswith("hbx"):
                print(f"{f.split('/')[-2]:8s} {k:28s} {c:26s} n={len(v):3d} avg={sum(v)/len(v):.6g}")

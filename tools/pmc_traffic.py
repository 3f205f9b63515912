#!/usr/bin/env python3
"""Turn a rocprofv3 FETCH_SIZE pass over bench.py into per-launch HBM bytes.

usage: python tools/pmc_traffic.py <counter_collection.csv> <out.json> [steps]

MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and, on gfx950, reads half the
bytes of a wide coalesced 16-B/lane stream, so hbm = 2 x FETCH_SIZE x 1024.
K1 (coalesced LDS-DMA landing) is that pattern; K3's cooperative loads (16
lanes x 16 B contiguous per chain) are the same width, its lane-mode loads are
not (flagged).  Per kernel the median over the steady-state dispatches (the
middle third of the run) is taken: K3 launches vary in size over the
pipeline's fill and drain.
"""
import collections
import csv
import json
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
by = collections.defaultdict(list)
for r in csv.DictReader(open(src)):
    if r["Counter_Name"] == "FETCH_SIZE" and r["Kernel_Name"].startswith("hbx_"):
        by[r["Kernel_Name"].split("(")[0]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
out = {"source": src, "formula": "2 x FETCH_SIZE[KiB] x 1024 (gfx950 wide-stream correction), "
                                  "median of the middle third of the dispatches", "kernels": {}}
for k, v in by.items():
    v.sort()
    mid = [x for _, x in v[len(v) // 3: 2 * len(v) // 3]] or [x for _, x in v]
    kib = statistics.median(mid)
    out["kernels"][k] = {"launches": len(v), "fetch_size_kib": kib, "hbm_bytes": 2.0 * kib * 1024.0,
                         "calibrated": k.startswith(("hbx_k1", "hbx_k3"))}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))

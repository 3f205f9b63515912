#!/usr/bin/env python3
"""Turn a rocprofv3 FETCH_SIZE pass into per-launch HBM bytes per kernel.

usage: python tools/pmc_traffic.py <counter_collection.csv> <out.json> [algorithmic_bytes]

MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and, on gfx950, reads exactly
half the bytes of a wide coalesced 16-B/lane stream, so
hbm_bytes = 2 x FETCH_SIZE x 1024 for such kernels (K1 after its coalesced
LDS-DMA landing).  K3's per-lane 64-B accesses are another width and are
uncalibrated; the same formula is applied and flagged.
"""
import collections
import csv
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
alg = float(sys.argv[3]) if len(sys.argv) > 3 else None
agg = collections.defaultdict(list)
for r in csv.DictReader(open(src)):
    if r["Counter_Name"] == "FETCH_SIZE" and r["Kernel_Name"].startswith("hbx_"):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
out = {"source": src, "formula": "2 x FETCH_SIZE[KiB] x 1024 (gfx950 wide-stream correction)",
       "kernels": {}}
for k, v in agg.items():
    fetch_kib = sum(v) / len(v)
    b = 2.0 * fetch_kib * 1024.0
    out["kernels"][k] = {"launches": len(v), "fetch_size_kib": fetch_kib, "hbm_bytes": b,
                         "calibrated": k.startswith("hbx_k1"),
                         "vs_algorithmic": (b / alg) if alg else None}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))

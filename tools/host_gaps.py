#!/usr/bin/env python3
"""Host side of the scan loop's long gaps: from a rocprofv3 run with
--kernel-trace and --hip-runtime-trace, for the K1 gaps longer than `min_us`,
the HIP API calls the host made between the end of one K1 and the start of
the next (name, start relative to the K1 end, duration), so a gap can be
charged to a host wait (hipEventSynchronize, ...) or to host work.

usage: python tools/host_gaps.py <trace dir> [min_us] [n_gaps]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
ngaps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
krows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
               for r in csv.DictReader(open(kt)))
hrows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Operation", "?")))
               for r in csv.DictReader(open(ht[0]))) if ht else []
k1 = [e for e in krows if e[2] in ("hbx_k1_digest_scan_dma", "hbx_k1d_digest_scan")]
shown = 0
for i in range(len(k1) - 1, 0, -1):
    a, b = k1[i - 1][1], k1[i][0]
    if (b - a) / 1e3 < min_us:
        continue
    print(f"-- K1 gap {(b - a) / 1e3:.1f} us")
    for s, e, name in hrows:
        if e >= a - 300_000 and s <= b:
            dur = (e - s) / 1e3
            if dur >= 5.0 or "Synchronize" in name or "Launch" in name:
                print(f"   {(s - a) / 1e3:9.1f} {dur:8.1f} us  {name}")
    shown += 1
    if shown >= ngaps:
        break

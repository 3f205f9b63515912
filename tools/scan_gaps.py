#!/usr/bin/env python3
"""Scan-loop gaps from a rocprofv3 trace: for the last `n` K1 launches, the
time from one K1's end to the next K1's start, and what ran on the GPU in
between (kernels, with their queue, and memory copies if a
memory_copy_trace.csv sits beside the kernel trace).

usage: python tools/scan_gaps.py <kernel_trace.csv> [n] [--show k]
"""
import csv
import glob
import os
import sys

import numpy as np

kt = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 100
show = int(sys.argv[sys.argv.index("--show") + 1]) if "--show" in sys.argv else 3
rows = list(csv.DictReader(open(kt)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
             r.get("Queue_Id", "")) for r in rows)
mc = glob.glob(os.path.join(os.path.dirname(kt), "*memory_copy_trace.csv"))
copies = []
if mc:
    for r in csv.DictReader(open(mc[0])):
        copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       f"copy {r.get('Direction', '')} {r.get('Bytes', r.get('Size', ''))}B", "dma"))
k1 = [e for e in ev if e[2] in ("hbx_k1_digest_scan_dma", "hbx_k1d_digest_scan")][-n:]
gaps = np.array([(k1[i + 1][0] - k1[i][1]) / 1e3 for i in range(len(k1) - 1)])
dur = np.array([(e - s) / 1e3 for s, e, _, _ in k1])
print(f"K1 launches {len(k1)}: duration us mean {dur.mean():.1f} median {np.median(dur):.1f}; "
      f"K1 end -> next K1 start us mean {gaps.mean():.1f} median {np.median(gaps):.1f} "
      f"p90 {np.percentile(gaps, 90):.1f} max {gaps.max():.1f}")
period = (k1[-1][0] - k1[0][0]) / 1e3 / (len(k1) - 1)
print(f"K1 start-to-start us {period:.1f}")
allev = sorted(ev + copies)
for i in list(range(len(k1) - 1))[-show:]:
    a, b = k1[i][1], k1[i + 1][0]
    print(f"-- gap {i}: {(b - a) / 1e3:.1f} us")
    for s, e, name, q in allev:
        if e >= a - 2000 and s <= b + 2000 and name != "hbx_k3p_block_md5":
            print(f"   {(s - a) / 1e3:9.1f} {(e - a) / 1e3:9.1f}  q{q:>3}  {name}")

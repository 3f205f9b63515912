#!/usr/bin/env python3
"""Per-step timeline of bench.py's timed window from a rocprofv3 kernel trace.

usage: python tools/window_timeline.py <kernel_trace.csv> <steps> [--all] [--seg a:b ...] [--lag L]

The bench (one workload, e.g. --workload random) ends with one drain K3
launch after the window, so the window holds the last `steps` K1 launches
and the `steps` K3 launches before the last.  For each window step: K1/K2
span on the scan stream, K3 span, the hash-stream gap before it and whether
the K3 waited for its batch's K2 (plan dependency).
"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2])


def spans(*names):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if r["Kernel_Name"].split("(")[0] in names)


LAG = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--lag=")), 1)  # drain launches after the window
k3 = spans("hbx_k3_block_md5", "hbx_k3p_block_md5", "hbx_k3q_block_md5")
k2 = spans("hbx_k2_cut_chain")
k1 = spans("hbx_k1_digest_scan_dma", "hbx_k1d_digest_scan", "hbx_k1_digest_scan_lite", "hbx_k1_digest_scan")
w3 = k3[-(K + LAG):-LAG]
w1 = k1[-K:]
w2 = k2[-K:]
t0 = w1[0][0]
ms = lambda x: x / 1e6  # noqa: E731
dur3 = np.array([ms(e - s) for s, e in w3])
gap = np.array([ms(w3[i][0] - w3[i - 1][1]) for i in range(1, K)])
span = ms(w3[-1][1] - t0)
print(f"window: first K1 start -> last K3 end {span:.2f} ms = {span / K:.3f} ms/step; "
      f"first K3 starts {ms(w3[0][0] - t0):.3f} ms after the first K1")
print(f"K3 ms: mean {dur3.mean():.3f} median {np.median(dur3):.3f} min {dur3.min():.3f} max {dur3.max():.3f}")
print(f"hash-stream gaps ms: sum {gap.sum():.2f} mean {gap.mean():.3f} max {gap.max():.3f}")
d1 = np.array([ms(e - s) for s, e in w1])
print(f"K1 ms: mean {d1.mean():.3f} first {d1[0]:.3f} max {d1.max():.3f}")
for arg in sys.argv[3:]:
    if arg.startswith("--seg="):
        a, b = (int(x) for x in arg[6:].split(":"))
        seg = ms(w3[b - 1][1] - w3[a][0]) / (b - a)
        print(f"steps {a}..{b}: {seg:.3f} ms/step  K3 mean {dur3[a:b].mean():.3f}  K1 mean {d1[a:b].mean():.3f}  "
              f"gaps {gap[max(a - 1, 0):b - 1].sum():.2f} ms  K1 start - K3 start mean "
              f"{np.mean([ms(w1[i][0] - w3[i][0]) for i in range(a, b)]):.3f}")
if "--all" in sys.argv or K <= 40:
    for i in range(K):
        wait = ms(w3[i][0] - w2[i][1])
        print(f"  step {i:3d}  K1 {ms(w1[i][0] - t0):8.3f}..{ms(w1[i][1] - t0):8.3f}  "
              f"K2 end {ms(w2[i][1] - t0):8.3f}  K3 {ms(w3[i][0] - t0):8.3f}..{ms(w3[i][1] - t0):8.3f} "
              f"({dur3[i]:.3f})  K3 start - K2 end {wait:7.3f}"
              + (f"  gap {gap[i - 1]:.3f}" if i else ""))

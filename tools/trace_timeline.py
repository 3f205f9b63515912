#!/usr/bin/env python3
"""Hash-stream timeline of bench.py's timed region from a rocprofv3 kernel trace.

usage: python tools/trace_timeline.py <run_kernel_trace.csv> [n_timed_k3]

For every timed K3 launch: its duration, the idle time on the hash stream
before the next K3 starts, and when the next batch's K2 (the plan's
dependency) ended relative to this K3's end.  A positive "K2 late" means the
hash stream waited for the scan stream.
"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))


def spans(name):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if r["Kernel_Name"].split("(")[0] == name)


k3 = spans("hbx_k3_block_md5")
k2 = spans("hbx_k2_cut_chain")
k1 = sorted(s for n in ("hbx_k1_digest_scan_dma", "hbx_k1_digest_scan_lite", "hbx_k1_digest_scan")
            for s in spans(n))
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(k3)
k3 = k3[-n:]
t0 = k3[0][0]
dur = np.array([(e - s) / 1e6 for s, e in k3])
gap = np.array([(k3[i + 1][0] - k3[i][1]) / 1e6 for i in range(len(k3) - 1)])
# the K2 that ends last before each K3 starts is the one its plan waited for
k2e = np.array([e for _, e in k2])
late = []
for i in range(len(k3) - 1):
    prev = k2e[k2e <= k3[i + 1][0]]
    if prev.size:
        late.append((prev.max() - k3[i][1]) / 1e6)
late = np.array(late)
k1d = np.array([(e - s) / 1e6 for s, e in k1 if s >= t0])
print(f"timed K3 launches: {len(k3)}  window {(k3[-1][1] - t0) / 1e6:.2f} ms")
print(f"K3 duration ms: median {np.median(dur):.3f} mean {dur.mean():.3f} "
      f"(w/o last {dur[:-1].mean():.3f}) max {dur.max():.3f} last {dur[-1]:.3f}")
print(f"hash-stream gap between K3s ms: median {np.median(gap):.3f} mean {gap.mean():.3f} "
      f"p90 {np.percentile(gap, 90):.3f} sum {gap.sum():.1f}")
if late.size:
    print(f"next batch's K2 end minus K3 end ms: median {np.median(late):.3f} mean {late.mean():.3f} "
          f"(>0, i.e. waited for the scan stream, in {int((late > 0).sum())} of {late.size})")
if k1d.size:
    print(f"K1 launch ms in window: median {np.median(k1d):.3f} mean {k1d.mean():.3f}")
mid = len(k3) // 2
for j in range(mid, min(mid + (6 if len(sys.argv) > 3 else 0), len(k3) - 1)):
    print(f"  k3[{j}] {(k3[j][0] - t0) / 1e6:9.3f} .. {(k3[j][1] - t0) / 1e6:9.3f}  "
          f"gap {(k3[j + 1][0] - k3[j][1]) / 1e6:.3f}")

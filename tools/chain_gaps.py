"""Dispatch gaps of the step's two loops, from a rocprofv3 kernel trace.

usage: python3 tools/chain_gaps.py <run_kernel_trace.csv> [...]

Per trace: the median gap between consecutive dispatches on the scan queue by
(kernel -> kernel) pair, the K3 -> K3 gap on the hash queue, the plan end ->
K3 start hop, and in how many launches the plan ended after the previous K3
(the scan-stream loop gate -> K1 -> K2 -> K2r -> plan was the later one; see
DESIGN.md §6 "two loops of equal length").
"""
import bisect
import csv
import statistics as st
import sys
from collections import defaultdict

SHORT = ["k1_gate", "k1_digest", "k2_cut", "k2r", "k2c_plan", "k3_block", "k4_content", "fillBuffer", "copyBuffer"]


def short(name):
    for k in SHORT:
        if k in name:
            return k
    return name[:20]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted(((short(r["Kernel_Name"]), int(r["Queue_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                 for r in rows), key=lambda e: e[2])
    k1q = next(e[1] for e in ev if e[0] == "k1_digest")
    scan = [e for e in ev if e[1] == k1q]
    gaps = defaultdict(list)
    for a, b in zip(scan, scan[1:]):
        gaps[(a[0], b[0])].append((b[2] - a[3]) / 1000)
    print(path)
    for k, v in sorted(gaps.items(), key=lambda x: -len(x[1])):
        if len(v) > 20:
            print(f"  scan {k[0]:>11s} -> {k[1]:<11s} n={len(v):4d} median {st.median(v):6.1f} us")
    k3 = [e for e in ev if e[0] == "k3_block"]
    pe = [e[3] for e in ev if e[0] == "k2c_plan"]
    hop, gap, late = [], [], 0
    for prev, cur in zip(k3, k3[1:]):
        i = bisect.bisect_right(pe, cur[2]) - 1
        if i < 0:
            continue
        hop.append((cur[2] - pe[i]) / 1000)
        gap.append((cur[2] - prev[3]) / 1000)
        late += pe[i] > prev[3]
    print(f"  K3 -> K3 gap median {st.median(gap):.1f} mean {st.mean(gap):.1f} us; plan end -> K3 start median "
          f"{st.median(hop):.1f} us; plan ended after the previous K3 in {late} of {len(gap)}")
    print(f"  K3 duration median {st.median([(e[3] - e[2]) / 1000 for e in k3]):.1f} us")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)

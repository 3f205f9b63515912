#!/usr/bin/env python3
"""Every kernel of a few pipeline steps from a rocprofv3 kernel trace, in
start order, relative to the first K3 shown (diagnostics: what sits between
two K3 launches on the hash stream).

usage: python tools/trace_steps.py <kernel_trace.csv> [first_k3_index] [n_k3]
(negative first_k3_index counts from the end)
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = int(sys.argv[2]) if len(sys.argv) > 2 else -20
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
             r.get("Queue_Id", r.get("Stream_Id", ""))) for r in rows)
k3 = [e for e in ev if e[2] in ("hbx_k3_block_md5", "hbx_k3p_block_md5", "hbx_k3q_block_md5")]
a, b = k3[first][0], k3[first + n][1] if first + n < 0 or first + n < len(k3) else k3[-1][1]
t0 = a
for s, e, name, q in ev:
    if e >= a and s <= b:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f}  q{q:>3}  {name}")

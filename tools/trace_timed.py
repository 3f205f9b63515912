#!/usr/bin/env python3
"""Per-kernel stats of bench.py's TIMED region from a rocprofv3 kernel trace.

usage: python tools/trace_timed.py <run_kernel_trace.csv> <bench.json line file>

rocprofv3 --stats averages every dispatch of the process, including the
untimed single-batch latency calls and the warm-up; bench.py's own numbers
cover only the timed steps.  The timed launches are the LAST n dispatches of
each kernel, n = the bench line's kernel_launches; this prints their average
next to bench.py's HIP-event average so the two can be compared.
"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
bench = None
for line in open(sys.argv[2]):
    if line.startswith("{") and '"metric"' in line:
        bench = json.loads(line)
names = {"k1_digest_scan": "hbx_k1_digest_scan_dma", "k2_cut_chain": "hbx_k2_cut_chain",
         "k2c_chain_plan": "hbx_k2c_plan", "k3_block_md5": "hbx_k3_block_md5",
         "k4_content_id": "hbx_k4_content_id"}
print(f"{'kernel':26s} {'timed n':>8s} {'rocprof avg ms':>15s} {'bench avg ms':>13s}")
for short, kern in names.items():
    d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
               if r["Kernel_Name"].split("(")[0] == kern)
    n = bench["kernel_launches"][short]
    timed = d[-n:]
    avg = sum(e - s for s, e in timed) / max(len(timed), 1) / 1e6
    bavg = bench["kernel_ms_per_step"][short] * bench["steps"] / max(n, 1)
    print(f"{kern:26s} {n:8d} {avg:15.4f} {bavg:13.4f}")

#!/usr/bin/env python3
"""Per-kernel stats of bench.py's TIMED region from a rocprofv3 kernel trace.

usage: python tools/trace_timed.py <run_kernel_trace.csv> <bench.json line file>

rocprofv3 --stats averages every dispatch of the process, including the
untimed single-batch latency calls and the warm-up; bench.py's own numbers
cover only the timed window (see below); this prints the window's rocprof
average next to bench.py's HIP-event average so the two can be compared.
"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
bench = None
for line in open(sys.argv[2]):
    if line.startswith("{") and '"metric"' in line:
        bench = json.loads(line)
names = {"k1_digest_scan": ("hbx_k1_digest_scan_dma", "hbx_k1d_digest_scan"), "k2_cut_chain": "hbx_k2_cut_chain",
         "k2c_chain_plan": "hbx_k2c_plan", "k3_block_md5": ("hbx_k3_block_md5", "hbx_k3p_block_md5", "hbx_k3q_block_md5"),
         "k4_content_id": "hbx_k4_content_id"}
# after the window, one drain launch per join-lag step (a preplanned launch
# plus each batch still unjoined): the window's K3 launches end that many early
lag = int(bench.get("config", {}).get("join_lag", 1))
print(f"{'kernel':26s} {'timed n':>8s} {'rocprof avg ms':>15s} {'bench avg ms':>13s}")
# the window (bench.py steady()): K1/K2 = the last n dispatches; K3 and its
# plan = the n before the final drain launch; K4 = dispatches starting inside
# [first window K1 start, last window K3 end]
launches = bench.get("window_launches") or bench["kernel_launches"]
spans = {k: sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                   if r["Kernel_Name"].split("(")[0] in ((v,) if isinstance(v, str) else v))
         for k, v in names.items()}
n1 = launches["k1_digest_scan"]
t_a = spans["k1_digest_scan"][-n1][0]
t_b = spans["k3_block_md5"][-(lag + 1)][1]
for short, kern in names.items():
    d = spans[short]
    n = launches[short]
    if short in ("k1_digest_scan", "k2_cut_chain"):
        timed = d[-n:]
    elif short in ("k3_block_md5", "k2c_chain_plan"):
        timed = d[-(n + lag):-lag]
    else:
        timed = [x for x in d if t_a <= x[0] <= t_b]
    avg = sum(e - s for s, e in timed) / max(len(timed), 1) / 1e6
    bavg = bench["kernel_ms_per_step"][short] * bench["steps"] / max(n, 1)
    kn = kern if isinstance(kern, str) else "/".join(sorted({r["Kernel_Name"].split("(")[0] for r in rows
                                                             if r["Kernel_Name"].split("(")[0] in kern}))
    print(f"{kn:26s} {len(timed):8d} {avg:15.4f} {bavg:13.4f}")

"""Median per-dispatch counters of the steady-state K3 launches (middle third
of the run) plus derived ratios.  usage: python tools/pmc_k3_summary.py <dir>"""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1]
per = collections.defaultdict(dict)  # (kernel, dispatch) -> counters
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], f.split("/")[-2], int(r["Dispatch_Id"]))
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        per[k]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
groups = collections.defaultdict(list)
for (kern, tag, disp), v in sorted(per.items()):
    groups[(kern, tag)].append(v)
agg = collections.defaultdict(dict)
for (kern, tag), rows in groups.items():
    mid = rows[len(rows) // 3: 2 * len(rows) // 3] or rows
    for c in set().union(*[r.keys() for r in mid]):
        vals = [r[c] for r in mid if c in r]
        agg[kern][c + ("" if c != "_ns" else "@" + tag)] = statistics.median(vals)
for kern, v in agg.items():
    print(kern)
    for c in sorted(v):
        print(f"   {c:40s} {v[c]:.6g}")
    g = lambda c: v.get(c, float("nan"))
    wc = g("SQ_WAVE_CYCLES")
    print(f"   wait_any/wave_cycles {g('SQ_WAIT_ANY') / wc:.3f}  active/wave_cycles {g('SQ_ACTIVE_INST_ANY') / wc:.3f}"
          f"  quad-cycles per VALU {wc / g('SQ_INSTS_VALU'):.3f}  waves {g('SQ_WAVES'):.0f}")
    print(f"   utcl1 miss rate {g('TCP_UTCL1_TRANSLATION_MISS_sum') / (g('TCP_UTCL1_TRANSLATION_MISS_sum') + g('TCP_UTCL1_TRANSLATION_HIT_sum')):.3f}"
          f"  tcp latency/instr {g('TCP_TCP_LATENCY_sum') / g('TCP_TA_TCP_STATE_READ_sum'):.0f} cyc")

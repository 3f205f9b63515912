#!/usr/bin/env python3
"""Which CUs end K3 launches late, launch after launch?  Runs bench.py's
default schedule (64 x 128 MiB, join lag 2) with the K3 probe on and reads
the per-wave records after every step (hbx_k3_wave_times syncs the hash
stream, so the pipeline is perturbed a little), then prints, per launch, the
median full-slice wave end, the launch span and the slowest CUs (XCC, SE, CU),
and over all launches how often each CU was among the slowest 8 waves.

Run on the GPU box: python tools/diag_slow_cu.py [--steps 30]"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import bench
    import workloads as W
    from hashbox_amd import Engine
    dev = torch.device("cuda", 0)
    free, _ = torch.cuda.mem_get_info(dev)
    P = bench.residency_plan(64, 128, 1, 0, "strong", free, 0.95)
    lens, offs, R, B, lag = P["lens"], P["offs"], P["R"], P["B"], P["join_lag"]
    arenas = W.random_arenas(R, P["arena_bytes"], 1000, dev)
    eng = Engine(0, md5_slice=B, join_lag=lag)
    eng.reserve(R + 2, len(lens), sum(lens))
    eng.set_k3_probe(True)
    count = collections.Counter()
    slowest_partial = collections.Counter()  # is each launch's last wave a partial (R < B) group?
    rows = []
    j = 0
    for _ in range(R):
        eng.submit_device(arenas[j % R].data_ptr(), offs, lens)
        j += 1
    for step in range(a.steps):
        eng.input_after_oldest()
        eng.submit_device(arenas[j % R].data_ptr(), offs, lens)
        j += 1
        eng.wait()
        w = eng.k3_wave_times().astype(np.int64)
        low56 = (1 << 56) - 1
        busy = w[(w[:, 1] & low56) != 0]
        t0 = int(w[w[:, 0] != 0][:, 0].min())
        end = (busy[:, 2] - t0) * 0.01
        Rw = busy[:, 3] & 0xffff
        full = Rw == Rw.max()
        hw = busy[:, 3] >> 32
        cu = [(int(x), int((h >> 13) & 3), int((h >> 8) & 0xf)) for x, h in zip(busy[:, 1] >> 56, hw)]
        order = np.argsort(-end)
        slow = [cu[i] for i in order[:8]]
        for c in set(slow):
            count[c] += 1
        # the first group's cooperative phase: cycles per block and the clock
        # (s_memtime cycles over s_memrealtime ticks), slowest waves vs median
        cyc = (busy[:, 5] - busy[:, 4]).astype(np.float64)
        ticks = (busy[:, 6] - (busy[:, 1] & low56)).astype(np.float64)
        nb = (busy[:, 7] & 0xffffffff).astype(np.float64)
        polls = (busy[:, 7] >> 32).astype(np.int64)  # stage-wait polls over the launch (s_sleep 1 each)
        ok = nb > 0
        cpb = np.where(ok, cyc / np.maximum(nb, 1), np.nan)
        ghz = np.where(ok, cyc / np.maximum(ticks, 1) * 0.1, np.nan)
        rows.append({"step": step, "median_full_end_us": round(float(np.median(end[full])), 1),
                     "span_us": round(float(end.max()), 1),
                     "median_cpb": round(float(np.nanmedian(cpb)), 1), "median_ghz": round(float(np.nanmedian(ghz)), 3),
                     "median_polls": float(np.median(polls[full])),
                     "slowest": [{"cu": cu[i], "end_us": round(float(end[i]), 1),
                                  "cpb": None if np.isnan(cpb[i]) else round(float(cpb[i]), 1),
                                  "ghz": None if np.isnan(ghz[i]) else round(float(ghz[i]), 3),
                                  "polls": int(polls[i]), "R": int(Rw[i]), "full": bool(full[i])}
                                 for i in order[:6]]})
        slowest_partial[bool(not full[order[0]])] += 1
        print(json.dumps(rows[-1]), flush=True)
    while eng.pending():
        eng.wait()
    print(json.dumps({"cu_in_slowest8_count": {str(k): v for k, v in count.most_common(12)},
                      "last_wave_partial_launches": slowest_partial[True],
                      "last_wave_full_launches": slowest_partial[False]}))
    eng.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""BASELINE config 1: one 1 GiB file (uniform random, PCG64 seed 1) through
storeFile's split + block hash.

GPU: (a) device-resident (file already in HBM, hbx_chunk_hash_device), (b)
from host memory (hbx_chunk_hash: H2D included).  CPU beside it: the
oracle's literal storeFile loop on ONE core (the reference runs storeFile on
one goroutine).  Cut lists and block IDs are compared bit-exact.

Run on the GPU box:  python tools/bench_config1.py      Prints one JSON line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from hashbox_amd import Engine, pack_arena_layout
    from oracle import oracle as O
    n = 1 << 30
    x = O.random_bytes(n, 1)
    eng = Engine(0)
    offs, total = pack_arena_layout([n])
    dev = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
    dev[:n].copy_(torch.from_numpy(x))
    torch.cuda.synchronize()
    eng.chunk_hash_device(dev.data_ptr(), offs, [n])  # warm-up
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        g_dev = eng.chunk_hash_device(dev.data_ptr(), offs, [n])[0]
    t_dev = (time.perf_counter() - t0) / reps
    st = eng.stage_times()
    t0 = time.perf_counter()
    g_host = eng.chunk_hash(x)
    t_host = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref = O.store_file(x)  # literal loop, one core
    t_cpu = time.perf_counter() - t0
    ok = all(np.array_equal(g.cut_ends, ref.cut_ends) and np.array_equal(g.ids, ref.ids)
             and g.content_id == ref.content_id for g in (g_dev, g_host))
    print(json.dumps({
        "config": "BASELINE configs[0]: one 1 GiB file, uniform random (PCG64 seed 1)",
        "chunks": int(ref.n_chunks), "longest_chunk": int(np.max(np.diff(np.concatenate([[0], ref.cut_ends])))),
        "bit_exact": bool(ok),
        "gpu_device_resident_s": round(t_dev, 4), "gpu_device_resident_gibs": round(1 / t_dev, 2),
        "gpu_stage_ms": [round(float(v), 3) for v in st],
        "gpu_from_host_s": round(t_host, 4), "gpu_from_host_gibs": round(1 / t_host, 2),
        "cpu_oracle_1core_s": round(t_cpu, 3), "cpu_oracle_1core_gibs": round(1 / t_cpu, 3),
        "note": "one file = one serial cut chain and MD5 chains of <= 8 MiB: latency-bound "
                "(longest chunk's MD5), not throughput-bound"}), flush=True)


if __name__ == "__main__":
    main()

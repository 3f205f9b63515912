#!/usr/bin/env python3
"""BASELINE config 4: 32 GiB Zipf-duplicated corpus (~50 % repeat content) —
bit-exact chunk boundaries and block IDs of the device path vs the CPU oracle.

Corpus: 256 files x 128 MiB built from random segments of 64 KiB-4 MiB.  Each
draw takes a fresh segment with probability 1/2, otherwise re-uses an earlier
one chosen by Zipf(1.1) rank (rank 1 = first used); the measured repeat
fraction (bytes of 2nd+ occurrences / total) is reported.  The corpus is built
on the device (torch), hashed in HBM by the engine, copied to host and checked
chunk by chunk against the oracle's literal storeFile loop on all host threads.

Run on the GPU box:  python tools/validate_config4.py [--gib 32] [--threads 16]
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def build_corpus(total, files, seed, dev):
    g = np.random.Generator(np.random.PCG64(seed))
    tg = torch.Generator(device=dev)
    tg.manual_seed(seed)
    arena = torch.empty(total + 65536, dtype=torch.uint8, device=dev)
    segs = []  # (offset in arena of first occurrence, size)
    pos = 0
    repeat = 0
    while pos < total:
        if not segs or g.random() < 0.5:
            size = int(g.integers(64 * 1024, 4 * 1024 * 1024 + 1))
            size = min(size, total - pos)
            arena[pos:pos + size].random_(0, 256, generator=tg)
            segs.append((pos, size))
        else:
            r = int(min(g.zipf(1.1), len(segs))) - 1
            src, size = segs[r]
            size = min(size, total - pos)
            arena[pos:pos + size].copy_(arena[src:src + size])
            repeat += size
        pos += size
    torch.cuda.synchronize()
    return arena, repeat / total, len(segs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=32)
    ap.add_argument("--files", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seed", type=int, default=4)
    a = ap.parse_args()
    from hashbox_amd import Engine
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    total = a.gib << 30
    fbytes = total // a.files
    t0 = time.time()
    arena, rep, nseg = build_corpus(total, a.files, a.seed, dev)
    t_build = time.time() - t0
    offs = np.arange(a.files, dtype=np.uint64) * np.uint64(fbytes)
    lens = [fbytes] * a.files
    eng = Engine(0)
    eng.chunk_hash_device(arena.data_ptr(), offs, lens)  # warm-up
    t0 = time.time()
    res = eng.chunk_hash_device(arena.data_ptr(), offs, lens)
    t_gpu = time.time() - t0
    st = eng.stage_times()
    # the same corpus again through the pipelined path: batches of 64 files
    # in flight together, time-sliced K3 (chains resume across launches)
    pipe = Engine(0, md5_slice=2048)
    per = max(1, a.files // 4)
    for b0 in range(0, a.files, per):
        pipe.submit_device(arena.data_ptr(), offs[b0:b0 + per], lens[b0:b0 + per])
    res_pipe = []
    while pipe.pending():
        res_pipe.extend(pipe.wait())
    pipe.close()
    host = arena[:total].cpu().numpy()
    files = [host[i * fbytes:(i + 1) * fbytes] for i in range(a.files)]
    t0 = time.time()
    ref = O.store_batch_mt(files, a.threads)
    t_cpu = time.time() - t0
    bad_cuts = bad_ids = 0
    n_chunks = 0
    pipe_bad = 0
    for g, gp, r in zip(res, res_pipe, ref):
        n_chunks += r.n_chunks
        if not np.array_equal(g.cut_ends, r.cut_ends):
            bad_cuts += 1
        elif not np.array_equal(g.ids, r.ids):
            bad_ids += 1
        if not (np.array_equal(gp.cut_ends, r.cut_ends) and np.array_equal(gp.ids, r.ids)
                and gp.content_id == g.content_id and gp.content_type == g.content_type):
            pipe_bad += 1
    print(json.dumps({
        "config": "BASELINE configs[3]: Zipf-duplicated corpus, bit-exactness vs oracle",
        "bytes": total, "files": a.files, "segments": nseg, "repeat_fraction": round(rep, 4),
        "chunks": n_chunks, "files_cut_mismatch": bad_cuts, "files_id_mismatch": bad_ids,
        "bit_exact": bad_cuts == 0 and bad_ids == 0 and pipe_bad == 0 and len(res_pipe) == a.files,
        "pipelined_files_mismatch": pipe_bad,
        "gpu_seconds": round(t_gpu, 4), "gpu_gibs": round(a.gib / t_gpu, 2),
        "gpu_stage_ms": [round(float(x), 3) for x in st],
        "cpu_oracle_seconds": round(t_cpu, 2), "cpu_threads": a.threads,
        "cpu_gibs": round(a.gib / t_cpu, 3), "build_seconds": round(t_build, 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Batch VerifyBlock throughput: the chunks of one configs[1]
batch (64 x 128 MiB random, ~2,050 chunks of 64 KiB - 8 MiB) re-verified
device-resident with hbx_verify_blocks_device, and a many-small-blocks case
(16,384 blocks of 4-64 KiB with 0-3 links).  Spot-checks against the oracle.
Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hashbox_amd import Engine, pack_arena_layout  # noqa: E402
from oracle import oracle as O  # noqa: E402

GIB = 1 << 30


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        best = min(best, time.perf_counter() - t0)
    return best, r


def main():
    O.lib()
    eng = Engine(0)
    nf, fb = 64, 128 << 20
    offs, total = pack_arena_layout([fb] * nf)
    arena = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1000)
    arena.random_(0, 256, generator=g)
    res = eng.chunk_hash_device(arena.data_ptr(), offs, [fb] * nf)
    c_offs, c_lens, expect = [], [], []
    for f, r in enumerate(res):
        s = 0
        for e, i in zip(r.cut_ends, r.ids):
            c_offs.append(int(offs[f]) + s)
            c_lens.append(int(e) - s)
            expect.append(i.tobytes())
            s = int(e)
    big_bytes = sum(c_lens)
    t_big, (ids, ok, bad) = timed(lambda: eng.verify_blocks_device(arena.data_ptr(), c_offs, c_lens,
                                                                    expect=expect))
    assert bad == 0 and ok.all()
    # many small blocks with links
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.integers(4096, 65536, 16384)]
    s_offs, s_total = pack_arena_layout(sizes)
    links = [[rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(int(k))]
             for k in rng.integers(0, 4, len(sizes))]
    small = torch.empty(s_total, dtype=torch.uint8, device="cuda:0")
    small.random_(0, 256, generator=g)
    host = small.cpu().numpy()
    sample = list(range(0, len(sizes), 97))
    exp_small = [O.block_id(host[int(s_offs[i]):int(s_offs[i]) + sizes[i]], links[i]) for i in sample]
    t_small, (ids_s, _, _) = timed(lambda: eng.verify_blocks_device(small.data_ptr(), s_offs, sizes, links))
    assert all(ids_s[i].tobytes() == e for i, e in zip(sample, exp_small))
    out = {
        "metric": "batch VerifyBlock GiB/s, device-resident (hbx_verify_blocks_device, K6)",
        "chunks_of_one_batch": {"blocks": len(c_lens), "bytes": big_bytes, "seconds": round(t_big, 4),
                                "gibs": round(big_bytes / t_big / GIB, 2),
                                "longest_block": max(c_lens)},
        "small_blocks": {"blocks": len(sizes), "bytes": sum(sizes), "seconds": round(t_small, 4),
                         "gibs": round(sum(sizes) / t_small / GIB, 2),
                         "blocks_per_s": round(len(sizes) / t_small)},
        "oracle_checked": {"chunks": "all (expect ids from the chunking path)", "small": len(sample)},
    }
    del arena, small
    torch.cuda.empty_cache()
    out["pipelined"] = pipelined(eng, nf, fb)
    print(json.dumps(out), flush=True)
    eng.close()


def pipelined(eng, nf, fb, steps=200, lead=2):
    """hbx_verify_submit_device over R distinct resident batches (the bench's
    residency rule: a batch's arena is reused only after its verify batch is
    collected), B = ceil(131073 / (R - lead)) blocks per chain per launch."""
    free, _ = torch.cuda.mem_get_info()
    per = nf * fb + (64 << 20)
    R = max(lead + 1, min(33, int(free * 0.90) // per))
    arenas, lists = [], []
    g = torch.Generator(device="cuda:0")
    for r in range(R):
        offs, total = pack_arena_layout([fb] * nf)
        a = torch.empty(total, dtype=torch.uint8, device="cuda:0")
        g.manual_seed(2000 + r)
        a.random_(0, 256, generator=g)
        torch.cuda.synchronize()
        res = eng.chunk_hash_device(a.data_ptr(), offs, [fb] * nf)
        co, cl, ex = [], [], []
        for f, rr in enumerate(res):
            s0 = 0
            for e, i in zip(rr.cut_ends, rr.ids):
                co.append(int(offs[f]) + s0)
                cl.append(int(e) - s0)
                ex.append(i.tobytes())
                s0 = int(e)
        arenas.append(a)
        lists.append((co, cl, ex))
    B = -(-131073 // (R - lead))
    pe = Engine(0, md5_slice=B)
    # a batch's chains join the K3 launch of the next submit (join lag 1) and
    # need ceil(131073 / B) launches: collect only once that many submits
    # have followed, or hbx_wait forces a drain launch (R - lead + 1 deep;
    # the arena of batch j is reused at submit j + R, after its collect)
    depth = -(-131073 // B) + 1
    bad = 0
    nbytes = 0

    def run(k):
        nonlocal bad, nbytes
        for j in range(k):
            if pe.pending() >= depth:
                bad += pe.wait()[2]
            co, cl, ex = lists[j % R]
            pe.verify_submit_device(arenas[j % R].data_ptr(), co, cl, expect=ex)
            nbytes += sum(cl)
        while pe.pending():
            bad += pe.wait()[2]

    run(min(R, 8))  # warm-up
    bad, nbytes = 0, 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    pe.close()
    return {"batches": steps, "resident_batches": R, "md5_slice_blocks": B, "bytes": nbytes,
            "seconds": round(dt, 3), "gibs": round(nbytes / dt / GIB, 2), "mismatches": int(bad),
            "note": "every chunk of every batch verified against the ids of the chunking path"}


if __name__ == "__main__":
    main()

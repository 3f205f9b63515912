#!/usr/bin/env python3
"""Diagnostic: pipelined results (several batches submitted back to back,
then drained) vs the synchronous path, on large random files."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hashbox_amd import Engine  # noqa: E402


def main():
    fb = 128 << 20
    for nb, per, sl in [(4, 16, 2048), (4, 16, 0), (1, 16, 2048), (2, 8, 2048)]:
        nf = nb * per
        arena = torch.empty(nf * fb + 65536, dtype=torch.uint8, device="cuda:0")
        g = torch.Generator(device="cuda:0")
        g.manual_seed(7)
        arena.random_(0, 256, generator=g)
        torch.cuda.synchronize()  # the engine's streams do not order after torch's
        offs = np.arange(nf, dtype=np.uint64) * np.uint64(fb)
        lens = [fb] * nf
        with Engine(0) as e:
            ref = e.chunk_hash_device(arena.data_ptr(), offs, lens)
        with Engine(0, md5_slice=sl) as p:
            for b0 in range(0, nf, per):
                p.submit_device(arena.data_ptr(), offs[b0:b0 + per], lens[b0:b0 + per])
            got = []
            while p.pending():
                got.extend(p.wait())
        bad_c = sum(not np.array_equal(a.cut_ends, b.cut_ends) for a, b in zip(got, ref))
        bad_i = sum(not np.array_equal(a.ids, b.ids) for a, b in zip(got, ref))
        bad_first = []
        for fi, (a, b) in enumerate(zip(got, ref)):
            if not np.array_equal(a.cut_ends, b.cut_ends):
                n = min(len(a.cut_ends), len(b.cut_ends))
                d = int(np.argmax(a.cut_ends[:n] != b.cut_ends[:n])) if (a.cut_ends[:n] != b.cut_ends[:n]).any() else n
                bad_first.append((fi, "cut", d, a.cut_ends[max(0, d - 1):d + 2].tolist(), b.cut_ends[max(0, d - 1):d + 2].tolist()))
            elif not np.array_equal(a.ids, b.ids):
                bad_first.append((fi, "id", int((a.ids != b.ids).any(axis=1).argmax())))
        print(f"batches {nb} x {per} files, slice {sl}: files {len(got)}, cut mismatches {bad_c}, "
              f"id mismatches {bad_i}, first bad {bad_first[:6]}", flush=True)
        del arena


if __name__ == "__main__":
    main()

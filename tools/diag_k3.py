"""Dev diagnostic: wave-mode (long chunks) and lane-mode block ids vs oracle."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hashbox_amd import Engine
from oracle import oracle as O

e = Engine(0)
for n in [300_000, 1 << 20, 8 * 1024 * 1024 - 1, 40_000_000]:
    x = O.random_bytes(n, 11)
    t = time.time()
    g = e.chunk_hash(x)
    dt = time.time() - t
    r = O.store_file(x, fast=True)
    bad = [i for i in range(min(g.n_chunks, r.n_chunks)) if g.ids[i].tobytes() != r.ids[i].tobytes()]
    print(n, "cuts_ok", np.array_equal(g.cut_ends, r.cut_ends), "nchunks", g.n_chunks, "bad", bad, f"{dt:.3f}s", e.stage_times().round(3), flush=True)

"""Dev diagnostic: which block IDs differ between the device and the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hashbox_amd import Engine
from oracle import oracle as O

e = Engine(0)
print("k5 hello", e.block_id(b"hello").hex(), O.py_block_id(b"hello").hex())
print("k5 64B", e.block_id(bytes(range(64))).hex(), O.py_block_id(bytes(range(64))).hex())
for n in [5, 40, 56, 57, 100, 1000, 5000, 70000, 200000, 3 * 1024 * 1024 + 12345]:
    x = O.random_bytes(n, 11)
    g = e.chunk_hash(x)
    r = O.store_file(x, fast=True)
    bad = [i for i in range(min(g.n_chunks, r.n_chunks)) if g.ids[i].tobytes() != r.ids[i].tobytes()]
    print(n, "cuts_ok", np.array_equal(g.cut_ends, r.cut_ends), "bad", bad, g.ids[0].tobytes().hex(), r.ids[0].tobytes().hex())

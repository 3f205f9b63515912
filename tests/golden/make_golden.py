#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.json).

Sources of truth, in order of strength:
  * kat.json — known answers that do not depend on this repo's code:
      - HMAC-MD5 vectors copied as DATA from the reference's own test
        pkg/core/core_test.go:23-30 (they pin the MD5 primitive);
      - BlockID("hello") = MD5(BE32(0)|BE32(5)|"hello") computed with Python
        hashlib, plus hashlib block ids for a few
        framing edge sizes.
  * chunking.json — storeFile results (hashback/store.go:111-196) for seeded
    synthetic inputs, computed by the C oracle's LITERAL loop and, for the
    inputs small enough, re-checked against the pure-Python transliteration
    and hashlib.  Inputs are not stored: they are regenerated from
    (kind, seed, n) by oracle.oracle's generators (numpy PCG64).  The
    rollsum arithmetic is assumption A1 (librsync rollsum; smtc/rollsum is
    absent from the image): these cut points are "oracle-consistent,
    reference-unpinned" except the constant-byte cases, whose cuts hold for
    ANY window-only digest.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

MIN = O.MIN_BLOCK_SIZE
MAXB = O.MAX_BLOCK_SIZE

# pkg/core/core_test.go:23-30 (out, depth, key, text)
HMAC_KATS = [
    ("74e6f7298a9c2d168935f58c001bad88", 1, "", ""),
    ("750c783e6ab0b503eaa86e310a5db738", 1, "Jefe", "what do ya want for nothing?"),
    ("80070713463e7749b90c2dc24911e275", 1, "key", "The quick brown fox jumps over the lazy dog"),
    ("64139538fd1a40dae8c3f99324f1f9a9", 20, "", ""),
    ("36b3f7b29692fbbf076d4cce1f9bbd2f", 20, "Jefe", "what do ya want for nothing?"),
    ("56881e862a44cbf94e92c5bf0bdbc497", 20, "key", "The quick brown fox jumps over the lazy dog"),
]


def make_input(case) -> np.ndarray:
    kind, seed, n = case["kind"], case["seed"], case["n"]
    if kind == "random":
        return O.random_bytes(n, seed)
    if kind == "const":
        return np.full(n, seed & 0xFF, np.uint8)
    if kind == "periodic":
        period = case["period"]
        base = O.random_bytes(period, seed)
        return np.resize(base, n)
    if kind == "zipf":
        return O.zipf_corpus(n, seed)
    raise ValueError(kind)


CASES = (
    [{"kind": "random", "seed": 1, "n": n} for n in
     [0, 1, 5, 55, 56, 63, 64, 65, 4096, MIN - 1, MIN, MIN + 1, 2 * MIN, 2 * MIN + 1,
      2 * MIN + 2, 200_000, 300_001]]
    + [{"kind": "random", "seed": s, "n": n} for s, n in
       [(2, 1 << 20), (3, 5 * MIN + 123), (4, MAXB - 1), (5, MAXB), (6, MAXB + 1),
        (7, MAXB + 2 * MIN + 1), (8, 3 * MAXB + 4321), (9, 40_000_000)]]
    + [{"kind": "const", "seed": v, "n": n} for v, n in [(0, 3 * MAXB + 777), (0x5A, MAXB + 5),
                                                         (255, 2 * MIN + 1)]]
    + [{"kind": "periodic", "seed": 10, "n": 21_000_000, "period": 70_001},
       {"kind": "periodic", "seed": 11, "n": 12_000_000, "period": 4096},
       {"kind": "zipf", "seed": 12, "n": 32 * 1024 * 1024}]
)


def block_id_hashlib(data: bytes) -> str:
    return hashlib.md5(struct.pack(">II", 0, len(data)) + data).hexdigest()


def main():
    kat = {
        "source": "HMAC rows: pkg/core/core_test.go:23-30; block ids: Python hashlib",
        "hmac": [{"out": o, "depth": d, "key": k, "text": t} for o, d, k, t in HMAC_KATS],
        "block_id": [{"data_hex": b"hello".hex(), "id": block_id_hashlib(b"hello")}],
    }
    for n in [0, 1, 55, 56, 57, 63, 64, 119, 120, 121, 1000]:
        d = bytes(O.random_bytes(n, 4242 + n))
        kat["block_id"].append({"data_hex": d.hex(), "id": block_id_hashlib(d)})
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)

    out = []
    for c in CASES:
        x = make_input(c)
        r = O.store_file(x)  # literal store.go loop
        rec = dict(c)
        rec["cut_ends"] = [int(v) for v in r.cut_ends]
        rec["ids"] = [bytes(i).hex() for i in r.ids]
        rec["content_type"] = r.content_type
        rec["content_id"] = r.content_id.hex()
        if x.size <= 400_000:  # independent re-check: Python loop + hashlib
            cuts, ids, ct, cid = O.py_store_file_literal(x.tobytes())
            assert cuts == rec["cut_ends"] and [i.hex() for i in ids] == rec["ids"]
            assert ct == rec["content_type"] and cid.hex() == rec["content_id"]
        else:  # hashlib re-check of every block id
            starts = [0] + rec["cut_ends"][:-1]
            for s, e, i in zip(starts, rec["cut_ends"], rec["ids"]):
                assert block_id_hashlib(x[s:e].tobytes()) == i
        out.append(rec)
        print(c["kind"], c["n"], len(rec["cut_ends"]), file=sys.stderr)
    with open(os.path.join(HERE, "chunking.json"), "w") as f:
        json.dump({"source": "oracle/hbx_oracle.c literal storeFile loop (assumption A1 rollsum); "
                             "regenerate inputs with tests/golden/make_golden.py:make_input",
                   "cases": out}, f, indent=0)


if __name__ == "__main__":
    main()

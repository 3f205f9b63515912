"""CPU: the oracle against known answers, the golden fixtures and itself.

The oracle (oracle/hbx_oracle.c) restates hashback/store.go:111-196 and
pkg/core/block.go:96-111; these tests pin it before it is trusted as the
checker of the GPU path.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_hmac_kats_from_reference_tests(oracle):
    # pkg/core/core_test.go:23-30 pins the MD5 primitive through HMAC-MD5
    for row in _load("kat.json")["hmac"]:
        got = oracle.hmac(row["text"].encode(), row["key"].encode(), row["depth"])
        assert got.hex() == row["out"]


def test_block_id_kats(oracle):
    for row in _load("kat.json")["block_id"]:
        d = bytes.fromhex(row["data_hex"])
        assert oracle.block_id(d).hex() == row["id"]
        assert oracle.py_block_id(d).hex() == row["id"]
    assert oracle.block_id(b"hello").hex() == "9e06002f060f42397d3862c8777fb39b"


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 127, 128, 1000, 4097, 100_000])
def test_md5_vs_hashlib(oracle, n):
    d = oracle.random_bytes(n, n + 3).tobytes()
    assert oracle.md5(d) == hashlib.md5(d).digest()


def test_block_id_with_links(oracle):
    links = [bytes(range(i, i + 16)) for i in range(3)]
    data = b"xyz" * 10
    ref = hashlib.md5(struct.pack(">I", 3) + b"".join(links) + struct.pack(">I", 30) + data)
    assert oracle.block_id(data, links) == ref.digest()
    assert oracle.py_block_id(data, links) == ref.digest()


def test_chain_id(oracle):
    ids = np.frombuffer(oracle.random_bytes(16 * 5, 9).tobytes(), np.uint8).reshape(5, 16)
    assert oracle.chain_id(ids) == oracle.py_chain_id([bytes(i) for i in ids])


def test_golden_chunking_fixtures(oracle):
    from tests.golden.make_golden import make_input
    for case in _load("chunking.json")["cases"]:
        if case["n"] > 48 * 1024 * 1024:
            continue
        x = make_input(case)
        r = oracle.store_file(x)
        assert [int(v) for v in r.cut_ends] == case["cut_ends"], case["kind"]
        assert [bytes(i).hex() for i in r.ids] == case["ids"]
        assert r.content_type == case["content_type"]
        assert r.content_id.hex() == case["content_id"]


@pytest.mark.parametrize("n,seed", [(131_073, 1), (200_000, 2), (250_001, 3)])
def test_c_literal_vs_python_literal(oracle, n, seed):
    x = oracle.random_bytes(n, seed)
    r = oracle.store_file(x)
    cuts, ids, ct, cid = oracle.py_store_file_literal(x.tobytes())
    assert [int(v) for v in r.cut_ends] == cuts
    assert [bytes(i) for i in r.ids] == ids
    assert r.content_type == ct and r.content_id == cid


@pytest.mark.parametrize("n,seed", [(5 * 65536 + 7, 4), (9 * 1024 * 1024, 5), (20_000_003, 6)])
def test_literal_vs_closed_form(oracle, n, seed):
    x = oracle.random_bytes(n, seed)
    a, b = oracle.store_file(x), oracle.store_file(x, fast=True)
    assert np.array_equal(a.cut_ends, b.cut_ends) and np.array_equal(a.ids, b.ids)


def test_window_digest_closed_form(oracle):
    # D[q] (closed form, virtual zeros) == Init + MIN Rollins + Digest of the window
    x = oracle.random_bytes(300_000, 8)
    D = oracle.digest_all(x)
    for q in [65535, 65536, 99_999, 299_999]:
        assert oracle.window_digest(x[q - 65535:q + 1]) == D[q]


def test_constant_bytes_cut_at_max(oracle):
    # tie rule ">=" (store.go:160): all digests equal -> cut at s+L
    x = np.full(2 * oracle.MAX_BLOCK_SIZE + 1000, 7, np.uint8)
    r = oracle.store_file(x)
    assert list(r.cut_ends) == [oracle.MAX_BLOCK_SIZE, 2 * oracle.MAX_BLOCK_SIZE, x.size]


def test_chunk_size_invariants(oracle):
    x = oracle.zipf_corpus(24 * 1024 * 1024, 3)
    r = oracle.store_file(x, fast=True)
    sizes = np.diff(np.concatenate([[0], r.cut_ends]).astype(np.int64))
    assert (sizes[:-1] >= oracle.MIN_BLOCK_SIZE).all()
    assert (sizes <= oracle.MAX_BLOCK_SIZE).all() and r.cut_ends[-1] == x.size


def test_batch_mt_matches_single(oracle):
    files = [oracle.random_bytes(n, 70 + n % 13) for n in [0, 5, 300_000, 3_000_000, 9_000_000]]
    got = oracle.store_batch_mt(files, 3)
    for f, g in zip(files, got):
        r = oracle.store_file(f)
        assert np.array_equal(g.cut_ends, r.cut_ends) and np.array_equal(g.ids, r.ids)

"""GPU parity of K1b (hbx_k1_digest_scan_dma2: 512 threads, 128-byte runs,
swizzled LDS image; HBX_K1_RUN=128) against the oracle's literal storeFile
loop (hashback/store.go:111-196), bit-exact: edge sizes in one batch, the
tie rule on constant and periodic bytes, K1 tile sizes (tile starts that
prime from the 64 KiB before them), a mixed batch, and the bench's
full-size steady-state schedule."""
import numpy as np
import pytest

from tests.test_gpu_parity import EDGE_SIZES, MAXB, MIN, _check

pytestmark = pytest.mark.gpu


@pytest.fixture
def k1b(monkeypatch):
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K1_RUN", "128")


def test_edge_sizes_batch(k1b, oracle):
    from hashbox_amd import Engine
    files = [oracle.random_bytes(n, 100 + n % 997) for n in EDGE_SIZES]
    with Engine(0) as e:
        got = e.chunk_hash_batch(files)
    for f, g in zip(files, got):
        _check(g, oracle.store_file(f, fast=True))


@pytest.mark.parametrize("val", [0, 0x5A, 255])
def test_constant_bytes(k1b, oracle, val):
    from hashbox_amd import Engine
    x = np.full(3 * MAXB + 777, val, np.uint8)
    with Engine(0) as e:
        _check(e.chunk_hash(x), oracle.store_file(x, fast=True))


def test_periodic_and_zipf(k1b, oracle):
    from hashbox_amd import Engine
    p = oracle.random_bytes(70001, 5)
    x = np.tile(p, 300)[: 20 * 1000 * 1000]
    z = oracle.zipf_corpus(48 * 1024 * 1024, 7)
    with Engine(0) as e:
        got = e.chunk_hash_batch([x, z])
    _check(got[0], oracle.store_file(x, fast=True))
    _check(got[1], oracle.store_file(z, fast=True))


@pytest.mark.parametrize("tile_iters", [1, 3, 32, 256])
def test_tile_sizes(k1b, oracle, tile_iters):
    from hashbox_amd import Engine
    n = 37 * MIN + 999 if tile_iters < 64 else (5 * tile_iters * MIN) // 2 + 999
    x = oracle.random_bytes(n, 77 + tile_iters)
    with Engine(0, tile_iters=tile_iters) as e:
        _check(e.chunk_hash(x), oracle.store_file(x, fast=True))


def test_batch_mixed(k1b, oracle):
    from hashbox_amd import Engine
    g = np.random.default_rng(19)
    sizes = [int(s) for s in np.exp(g.uniform(np.log(1), np.log(20e6), 60))] + [0, 1, 2 * MIN + 1]
    files = [oracle.random_bytes(n, 3000 + i) for i, n in enumerate(sizes)]
    with Engine(0) as e:
        got = e.chunk_hash_batch(files)
    for f, r in zip(files, got):
        _check(r, oracle.store_file(f, fast=True))


def test_full_size_steady_state(k1b, oracle):
    import torch
    import workloads as W
    from tests.test_gpu_fullsize import _check as check_full, _oracle_of, _run_schedule
    lens = [128 << 20] * 64
    offs, total = W.pack_layout(lens)
    arenas = W.random_arenas(2, total, 2024, torch.device("cuda", 0))
    refs = [_oracle_of(oracle, a, offs, lens) for a in arenas]
    results = _run_schedule(arenas, offs, lens, steps=36)
    check_full(results, refs)
    del arenas
    torch.cuda.empty_cache()

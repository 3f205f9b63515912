"""GPU parity of batched HashboxBlock.HashData / VerifyBlock:
libhbxgpu's K6 vs the oracle's restatement of pkg/core/block.go:96-111 (the
framing BE32(n_links) || links || BE32(len) || data), bit-exact, plus the
reference's own VerifyBlock failure cases (pkg/core/block_test.go:86-117).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# data lengths around the message-block edges for every prefix size class
# (prefix = 8 + 16 * n_links bytes: 8, 24, 40, 56, 72, ...)
LENS = [0, 1, 7, 8, 9, 40, 47, 48, 55, 56, 57, 63, 64, 65, 111, 119, 120, 121, 183, 184, 185,
        4096, 65536 + 17, 1 << 20]


def _rand_links(rng, k):
    return [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(k)]


def test_hello_known_answer(engine):
    ids, ok, bad = engine.verify_blocks([b"hello"], expect=[bytes.fromhex("9e06002f060f42397d3862c8777fb39b")])
    assert ids[0].tobytes().hex() == "9e06002f060f42397d3862c8777fb39b"
    assert ok.tolist() == [True] and bad == 0


@pytest.mark.parametrize("n_links", [0, 1, 2, 3, 4, 5, 9])
def test_ids_vs_oracle_edge_lengths(engine, oracle, n_links):
    rng = np.random.default_rng(1000 + n_links)
    blocks = [oracle.random_bytes(n, 7 * n + n_links) for n in LENS]
    links = [_rand_links(rng, n_links) for _ in LENS]
    ids, ok, bad = engine.verify_blocks(blocks, links)
    assert ok is None and bad == 0
    for b, l, got in zip(blocks, links, ids):
        assert got.tobytes() == oracle.block_id(b, l)


def test_mixed_batch_and_failures(engine, oracle):
    """Many blocks with mixed sizes and link counts in one call; the
    reference's failure cases: corrupted data (block_test.go:86-101) and
    tampered links (block_test.go:105-117) fail, everything else passes."""
    rng = np.random.default_rng(7)
    n = 700
    sizes = [int(x) for x in rng.integers(0, 300_000, n)]
    sizes[:5] = [0, 8 << 20, 3, 65536, 2 * 65536 + 1]
    blocks = [oracle.random_bytes(s, 50_000 + i) for i, s in enumerate(sizes)]
    links = [_rand_links(rng, int(k)) for k in rng.integers(0, 6, n)]
    expect = [oracle.block_id(b, l) for b, l in zip(blocks, links)]
    ids, ok, bad = engine.verify_blocks(blocks, links, expect)
    assert bad == 0 and ok.all()
    assert all(i.tobytes() == e for i, e in zip(ids, expect))
    # corrupt data of block 3, a link of block 10 (which has links), and the
    # expected id of block 20
    blocks[3] = blocks[3].copy()
    blocks[3][-1] ^= 1
    j = next(i for i in range(10, n) if links[i] and sizes[i])
    links[j] = [bytes([links[j][0][0] ^ 0x80]) + links[j][0][1:]] + links[j][1:]
    expect[20] = bytes(16)
    ids, ok, bad = engine.verify_blocks(blocks, links, expect)
    assert bad == 3 and not ok[3] and not ok[j] and not ok[20]
    assert ok.sum() == n - 3


def test_device_resident(engine, oracle):
    import torch
    from hashbox_amd import pack_arena_layout
    rng = np.random.default_rng(11)
    sizes = [int(x) for x in rng.integers(0, 2_000_000, 200)]
    blocks = [oracle.random_bytes(s, 90_000 + i) for i, s in enumerate(sizes)]
    links = [_rand_links(rng, int(k)) for k in rng.integers(0, 4, len(sizes))]
    offs, total = pack_arena_layout(sizes)
    host = np.zeros(total, np.uint8)
    for o, b in zip(offs, blocks):
        host[int(o):int(o) + b.size] = b
    dev = torch.from_numpy(host).to("cuda:0")
    expect = [oracle.block_id(b, l) for b, l in zip(blocks, links)]
    ids, ok, bad = engine.verify_blocks_device(dev.data_ptr(), offs, sizes, links, expect)
    assert bad == 0 and ok.all()
    assert [i.tobytes() for i in ids] == expect


@pytest.mark.parametrize("md5_slice,join_lag,period", [(0, 1, 1), (3, 1, 1), (256, 1, 1), (256, 3, 1), (3, 2, 1),
                                                       (256, 2, 3), (3, 3, 2)])
def test_pipelined_verify_with_chunking(oracle, md5_slice, join_lag, period):
    """hbx_verify_submit_device: verify batches share the time-sliced K3
    pipeline and the wait FIFO with chunking batches; every edge length for
    0-9 links, blocks past 8 MiB, expected-id mismatches; with a K3 period
    verify and chunking batches join one launch together."""
    import torch
    from hashbox_amd import Engine
    rng = np.random.default_rng(77 + md5_slice)
    lens = LENS + [(8 << 20) + 12345, 3 << 20]
    specs = [(n, k) for k in (0, 1, 2, 3, 5, 9) for n in lens]
    datas = [oracle.random_bytes(n, 31 * n + k + 1) for n, k in specs]
    links = [_rand_links(rng, k) for _, k in specs]
    want = [oracle.block_id(d, l) for d, l in zip(datas, links)]
    expect = list(want)
    for j in range(0, len(expect), 7):  # tampered expectations
        expect[j] = bytes(16) if expect[j] != bytes(16) else b"\x01" * 16
    offs, pos = [], 0
    for d in datas:
        offs.append(pos)
        pos += (d.size + 255) // 256 * 256 + 256
    host = np.zeros(pos + 65536, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + d.size] = d
    arena = torch.from_numpy(host).to("cuda:0")
    files = [oracle.random_bytes(3 << 20, 5), oracle.random_bytes(300_000, 6)]
    fhost = np.zeros((4 << 20) + 300_000 + 65536, np.uint8)
    fhost[:files[0].size] = files[0]
    fhost[4 << 20:(4 << 20) + files[1].size] = files[1]
    farena = torch.from_numpy(fhost).to("cuda:0")
    torch.cuda.synchronize()
    third = len(specs) // 3
    with Engine(0, md5_slice=md5_slice, join_lag=join_lag, k3_period=period) as eng:
        eng.verify_submit_device(arena.data_ptr(), offs[:third], [d.size for d in datas[:third]],
                                 links[:third], expect[:third])
        eng.submit_device(farena.data_ptr(), [0, 4 << 20], [f.size for f in files])
        eng.verify_submit_device(arena.data_ptr(), offs[third:], [d.size for d in datas[third:]],
                                 links[third:], expect[third:])
        eng.verify_submit_device(arena.data_ptr(), offs[:5], [d.size for d in datas[:5]])  # ids only
        r1 = eng.wait()
        rf = eng.wait()
        r2 = eng.wait()
        r3 = eng.wait()
        assert eng.pending() == 0
    ids = np.concatenate([r1[0], r2[0]])
    ok = np.concatenate([r1[1], r2[1]])
    for i in range(len(specs)):
        assert ids[i].tobytes() == want[i], (i, specs[i])
        assert bool(ok[i]) == (expect[i] == want[i])
    assert r1[2] + r2[2] == sum(e != w for e, w in zip(expect, want))
    assert r3[1] is None and all(r3[0][i].tobytes() == want[i] for i in range(5))
    for f, r in zip(files, rf):
        ref = oracle.store_file(f, fast=True)
        assert np.array_equal(r.cut_ends, ref.cut_ends) and np.array_equal(r.ids, ref.ids)

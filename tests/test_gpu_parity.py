"""GPU parity: libhbxgpu (HIP, gfx950) vs the CPU oracle, bit-exact.

Chunk boundaries, block IDs, content type and content ID must equal the
oracle's restatement of hashback/store.go:111-196 + pkg/core/block.go:96-111.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MIN = 65536
MAXB = 8 * 1024 * 1024


def _check(got, ref):
    assert np.array_equal(got.cut_ends, ref.cut_ends), (got.cut_ends[:8], ref.cut_ends[:8])
    assert np.array_equal(got.ids, ref.ids), "block ids differ"
    assert got.content_type == ref.content_type
    assert got.content_id == ref.content_id


def _check_mt(oracle, got, ref):
    """Against oracle.store_batch_mt (cut ends and block ids only): the content
    type and id follow store.go:187-196 (one chunk: its id; else the chain
    block's id, oracle chain_id)."""
    assert np.array_equal(got.cut_ends, ref.cut_ends), (got.cut_ends[:8], ref.cut_ends[:8])
    assert np.array_equal(got.ids, ref.ids), "block ids differ"
    k = ref.n_chunks
    assert got.content_type == (0 if k == 0 else 2 if k == 1 else 3)
    if k:
        assert got.content_id == (ref.ids[0].tobytes() if k == 1 else oracle.chain_id(ref.ids))


EDGE_SIZES = [0, 1, 5, 55, 56, 57, 63, 64, 65, 119, 120, 121, 4095, 4096, MIN - 1, MIN, MIN + 1,
              2 * MIN - 1, 2 * MIN, 2 * MIN + 1, 2 * MIN + 2, 3 * MIN + 17, MAXB - 1, MAXB,
              MAXB + 1, MAXB + 2 * MIN + 1, 2 * MAXB + 12345]


@pytest.mark.parametrize("n", EDGE_SIZES)
def test_edge_sizes_random(engine, oracle, n):
    x = oracle.random_bytes(n, 100 + n % 997)
    _check(engine.chunk_hash(x), oracle.store_file(x, fast=True))


def test_hello_known_answer(engine):
    r = engine.chunk_hash(b"hello")
    assert r.n_chunks == 1 and r.cut_ends[0] == 5
    assert r.ids[0].tobytes().hex() == "9e06002f060f42397d3862c8777fb39b"
    assert r.content_type == 2


def test_literal_oracle_small(engine, oracle):
    # the literal re-rolled loop (store.go:141-165) on a few sizes
    for n, seed in [(131073, 1), (200000, 2), (300001, 3), (1 << 20, 4)]:
        x = oracle.random_bytes(n, seed)
        _check(engine.chunk_hash(x), oracle.store_file(x, fast=False))


@pytest.mark.parametrize("val", [0, 0x5A, 255])
def test_constant_bytes_tie_rule(engine, oracle, val):
    # all digests equal -> ">=" keeps the LAST position -> 8 MiB chunks
    x = np.full(3 * MAXB + 777, val, np.uint8)
    r = engine.chunk_hash(x)
    assert list(r.cut_ends[:3]) == [MAXB, 2 * MAXB, 3 * MAXB]
    _check(r, oracle.store_file(x, fast=True))


def test_periodic_ties(engine, oracle):
    x = np.tile(oracle.random_bytes(70001, 5), 300)
    _check(engine.chunk_hash(x), oracle.store_file(x, fast=True))
    x = np.tile(oracle.random_bytes(4096, 6), 3000)  # period < window
    _check(engine.chunk_hash(x), oracle.store_file(x, fast=True))


@pytest.mark.parametrize("window", [1, 3, 16])
def test_content_id_windows(oracle, monkeypatch, window):
    """K4 stages a file's ids through an LDS window (1,024 ids; shrunk here
    with HBX_K4_WINDOW) and reads them twice, as ids and as links: files of
    many more chunks than the window restage it on both passes."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K4_WINDOW", str(window))
    files = [oracle.random_bytes(n, 60 + i) for i, n in enumerate([9 * MAXB + 3, 40 * MAXB + 11, 3 * MIN])]
    with Engine(0) as e:
        got = e.chunk_hash_batch(files)
    assert got[1].n_chunks > 3 * window
    for f, r in zip(files, got):
        _check(r, oracle.store_file(f, fast=True))


def test_zipf_duplicates(engine, oracle):
    x = oracle.zipf_corpus(48 * 1024 * 1024, 7)
    _check(engine.chunk_hash(x), oracle.store_file(x, fast=True))


def test_batch_mixed(engine, oracle):
    g = np.random.default_rng(9)
    sizes = [int(s) for s in np.exp(g.uniform(np.log(1), np.log(20e6), 60))] + [0, 1, 2 * MIN + 1]
    files = [oracle.random_bytes(n, 1000 + i) for i, n in enumerate(sizes)]
    got = engine.chunk_hash_batch(files)
    for f, r in zip(files, got):
        _check(r, oracle.store_file(f, fast=True))


@pytest.mark.parametrize("swz", ["0", "1"])
@pytest.mark.parametrize("tile_iters", [0, 1, 3, 32, 64, 256, 1024])
def test_tile_sizes(oracle, monkeypatch, tile_iters, swz):
    """K1 tiles of 1..1024 iterations; swz 1: the LDS image transposed per
    1 KiB (HBX_K1_SWZ), ragged file ends included."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K1_SWZ", swz)
    # several tiles per file up to 256 iterations (16 MiB tiles); 1024 = one
    # tile; 0 = sized per batch (16 iterations for this one)
    n = 37 * MIN + 999 if tile_iters < 64 else (5 * tile_iters * MIN) // 2 + 999 if tile_iters <= 256 else 20 * MAXB + 5
    with Engine(0, tile_iters=tile_iters) as e:
        assert e.knobs()["k1_swz"] == int(swz)
        x = oracle.random_bytes(n, 77)
        _check(e.chunk_hash(x), oracle.store_file(x, fast=True))
        y = oracle.random_bytes(n // 3 + 17, 78)
        _check(e.chunk_hash(y), oracle.store_file(y, fast=True))


def test_device_resident(engine, oracle):
    import torch
    from hashbox_amd import pack_arena_layout
    sizes = [5 * MAXB + 3, 129 * 1024, 7, 3 * MAXB]
    files = [oracle.random_bytes(n, 50 + i) for i, n in enumerate(sizes)]
    offs, total = pack_arena_layout(sizes)
    host = np.zeros(total, np.uint8)
    for o, f in zip(offs, files):
        host[int(o):int(o) + f.size] = f
    dev = torch.from_numpy(host).to("cuda:0")
    torch.cuda.synchronize()
    got = engine.chunk_hash_device(dev.data_ptr(), offs, sizes)
    for f, r in zip(files, got):
        _check(r, oracle.store_file(f, fast=True))
    # async submit/wait gives the same
    engine.submit_device(dev.data_ptr(), offs, sizes)
    got2 = engine.wait()
    for a, b in zip(got, got2):
        _check(a, b)


def test_block_id_with_links(engine, oracle):
    links = [bytes(range(i, i + 16)) for i in range(5)]
    data = b"fchn" + bytes(100)
    assert engine.block_id(data, links) == oracle.py_block_id(data, links)
    assert engine.block_id(b"") == oracle.py_block_id(b"")


def test_golden_fixtures_on_device(engine):
    """The committed fixtures (tests/golden/chunking.json) through the HIP path."""
    import json
    import os
    from tests.golden.make_golden import make_input
    with open(os.path.join(os.path.dirname(__file__), "golden", "chunking.json")) as f:
        cases = json.load(f)["cases"]
    xs = [make_input(c) for c in cases]
    got = engine.chunk_hash_batch(xs)
    for c, g in zip(cases, got):
        assert [int(v) for v in g.cut_ends] == c["cut_ends"], (c["kind"], c["n"])
        assert [bytes(i).hex() for i in g.ids] == c["ids"]
        assert g.content_type == c["content_type"] and g.content_id.hex() == c["content_id"]


def test_hmac_kats_on_device_md5(engine):
    """The reference's own HMAC-MD5 rows (pkg/core/core_test.go:23-30, kept in
    tests/golden/kat.json) computed with the device MD5 (hbx_md5, K5) as the
    hash under core.Hmac / DeepHmac: pins the GPU MD5 to the reference's
    vectors directly, not only through the oracle."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")) as f:
        kat = json.load(f)
    for r in kat["hmac"]:
        got = engine.deep_hmac(r["depth"], r["text"].encode(), r["key"].encode())
        assert got.hex() == r["out"], r


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 1000, 65536, 1 << 20])
def test_md5_raw_lengths(engine, n):
    """hbx_md5 against hashlib over the padding boundaries (55/56/64 mod 64)."""
    import hashlib
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    assert engine.md5(data) == hashlib.md5(data).digest()


def test_kat_block_ids_on_device(engine):
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")) as f:
        kat = json.load(f)
    datas = [bytes.fromhex(r["data_hex"]) for r in kat["block_id"]]
    got = engine.chunk_hash_batch(datas)  # each <= 2*MIN: one chunk = the block id
    for r, g in zip(kat["block_id"], got):
        assert g.ids[0].tobytes().hex() == r["id"] if g.n_chunks else r["data_hex"] == ""
        assert engine.block_id(bytes.fromhex(r["data_hex"])).hex() == r["id"]


@pytest.mark.parametrize("join_lag,period", [(1, 1), (3, 1), (2, 4)])
def test_store_paths_end_to_end(oracle, tmp_path, join_lag, period):
    """Files on disk -> pinned -> HBM -> results, in small batches so the
    two-stream double buffering and batch boundaries are exercised (the
    arena ring is as deep as the slice schedule plus the join lag, and the
    K3 period's extra submits)."""
    from hashbox_amd import Engine
    engine = Engine(0, md5_slice=4096, join_lag=join_lag, k3_period=period)
    sizes = [0, 1, 4096, 2 * MIN + 1, 3 * MAXB + 7, 700_001, 5 * MIN, 12345, 9 * 1024 * 1024]
    paths, datas = [], []
    for i, n in enumerate(sizes * 3):
        x = oracle.random_bytes(n, 900 + i)
        p = tmp_path / f"f{i:03d}.bin"
        p.write_bytes(x.tobytes())
        paths.append(str(p))
        datas.append(x)
    got = engine.store_paths(paths, io_threads=4, batch_bytes=64 << 20)
    for x, g in zip(datas, got):
        _check(g, oracle.store_file(x, fast=True))
    # a missing file fails loudly
    import pytest as _pt
    from hashbox_amd import HbxError
    with _pt.raises((HbxError, FileNotFoundError)):
        engine.store_paths([str(tmp_path / "missing.bin")])
    # the walker's sizes (FileEntry.FileSize) instead of a stat per path
    got = engine.store_paths(paths, io_threads=4, batch_bytes=64 << 20, sizes=[x.size for x in datas])
    for x, g in zip(datas, got):
        _check(g, oracle.store_file(x, fast=True))
    # a size past the end of the file fails loudly
    with _pt.raises(HbxError):
        engine.store_paths(paths[3:4], sizes=[datas[3].size + 1])
    with _pt.raises(ValueError):
        engine.store_paths(paths[:2], sizes=[1])
    engine.close()


@pytest.mark.parametrize("compress", [False, True])
def test_store_paths_per_file_status(engine, oracle, tmp_path, compress):
    """hbx_store_paths_status (verdict r04 item 5): one file of a 1,000-file
    batch cannot be opened (deleted after the walker's stat, ENOENT).  The
    reference's storeDir logs it and goes on (store.go:101-103, 221-224), so
    the call succeeds, that file gets no chunks and its errno, and the other
    999 are bit-exact.  A read error the reference panics on (a file shorter
    than its size, CopyNOrPanic utils.go:95-99; a directory) still fails the
    whole call."""
    import errno
    from hashbox_amd import HbxError
    g = np.random.Generator(np.random.PCG64(77))
    sizes = np.exp(g.uniform(np.log(1), np.log(3 << 20), 1000)).astype(np.int64)
    pool = g.integers(0, 256, 8 << 20, dtype=np.uint8)
    datas, paths = [], []
    for i, n in enumerate(sizes):
        o = int(g.integers(0, pool.size - int(n)))
        datas.append(pool[o:o + int(n)])
        p = tmp_path / f"s{i:04d}.bin"
        datas[-1].tofile(p)
        paths.append(str(p))
    bad = 471
    os.unlink(paths[bad])
    got = engine.store_paths(paths, sizes=sizes, batch_bytes=256 << 20, compress=compress, skip_unreadable=True)
    refs = oracle.store_batch_mt(datas, 16)
    for i, (r, gg) in enumerate(zip(refs, got)):
        if i == bad:
            assert gg.errno == errno.ENOENT and gg.n_chunks == 0 and gg.content_type == 0
            continue
        assert gg.errno == 0
        _check_mt(oracle, gg, r)
        if compress:
            assert len(gg.zstreams) == r.n_chunks
    # without per-file status the same batch fails loudly, naming the file
    with pytest.raises(HbxError, match=f"s{bad:04d}.bin"):
        engine.store_paths(paths, sizes=sizes, batch_bytes=256 << 20, compress=compress)
    # errors the reference panics on fail the call even with per-file status
    datas[bad].tofile(paths[bad])
    short = list(sizes)
    short[3] += 1
    with pytest.raises(HbxError, match="end of file"):
        engine.store_paths(paths, sizes=short, compress=compress, skip_unreadable=True)
    with pytest.raises(HbxError):
        engine.store_paths([str(tmp_path)] + paths[:2], sizes=[4096] + list(sizes[:2]), compress=compress,
                           skip_unreadable=True)
    # and the context is fine afterwards
    got = engine.store_paths(paths[:20], sizes=sizes[:20], compress=compress, skip_unreadable=True)
    for r, gg in zip(refs[:20], got):
        assert gg.errno == 0
        _check_mt(oracle, gg, r)


def _device_batches(oracle, nb, seed):
    """nb device-resident batches of mixed files (edge lengths, long chunks,
    constant runs) plus their oracle results."""
    import torch
    from hashbox_amd import pack_arena_layout
    rng = np.random.default_rng(seed)
    out = []
    for b in range(nb):
        sizes = [int(rng.integers(0, 3 * MAXB)) for _ in range(5)] + [0, 57, 2 * MIN + 1, MAXB + 9]
        files = [oracle.random_bytes(n, seed * 100 + 10 * b + i) for i, n in enumerate(sizes)]
        files[1] = np.full(sizes[1], 0x5A, np.uint8)  # constant run: 8 MiB max-length chunks
        offs, total = pack_arena_layout(sizes)
        host = np.zeros(total, np.uint8)
        for o, f in zip(offs, files):
            host[int(o):int(o) + f.size] = f
        dev = torch.from_numpy(host).to("cuda:0")
        out.append((dev, offs, sizes, [oracle.store_file(f, fast=True) for f in files]))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("md5_slice,join_lag", [(1, 1), (3, 1), (9, 1), (64, 1), (16384, 1), (3, 2), (64, 2), (64, 3),
                                                (16384, 4)])
def test_pipelined_batches_time_sliced(oracle, md5_slice, join_lag):
    """Several batches in flight on one context with the block-MD5 stage
    time-sliced: chains resume across many K3 launches, new batches' chunks
    join carried chains (join_lag submits later), results come back in FIFO
    order, bit-exact."""
    from hashbox_amd import Engine
    batches = _device_batches(oracle, 4, 31 + md5_slice % 7)
    with Engine(0, md5_slice=md5_slice, join_lag=join_lag) as e:
        for dev, offs, sizes, _ in batches[:3]:
            e.submit_device(dev.data_ptr(), offs, sizes)
        assert e.pending() == 3
        first = e.wait()  # may force a drain of every chain in flight
        e.submit_device(batches[3][0].data_ptr(), batches[3][1], batches[3][2])
        rest = [e.wait() for _ in range(3)]
        assert e.pending() == 0 and e.wait() == []
        for (_, _, _, ref), got in zip(batches, [first] + rest):
            for g, r in zip(got, ref):
                _check(g, r)
        # the synchronous path is refused while batches are pending
        from hashbox_amd import HbxError
        e.submit_device(batches[0][0].data_ptr(), batches[0][1], batches[0][2])
        with pytest.raises(HbxError):
            e.chunk_hash(b"x")
        for g, r in zip(e.wait(), batches[0][3]):
            _check(g, r)
        ms, n = e.stage_totals()
        assert n[3] >= 1 and ms[3] > 0


@pytest.mark.parametrize("prod", ["0", "1", "q2", "q4", "p3"])
@pytest.mark.parametrize("md5_slice,join_lag,wgs,plan_cut", [
    (9, 1, 0, "0"), (64, 3, 0, "0"), (4096, 1, 0, "0"), (4096, 2, 0, "0"), (16384, 1, 0, "0"), (0, 1, 0, "0"),
    (64, 1, 1, "0"), (4096, 1, 2, "0"), (0, 3, 1, "0"), (4096, 2, 0, "1"), (64, 2, 0, "1"), (9, 2, 1, "1"),
    (64, 3, 0, "2"), (4096, 4, 1, "2")])
def test_k3_producer_waves(oracle, monkeypatch, md5_slice, join_lag, wgs, plan_cut, prod):
    """K3 with and without a producer wave per MD5 wave (hbx_k3p_block_md5 /
    hbx_k3_block_md5, HBX_K3_PROD): the stages a producer hands over through
    the LDS counters, groups on the lane path (slices below 8 blocks), groups
    that straddle two bins (partial rounds self-staged in the same LDS), many
    groups per wave (more groups than waves at small slices), a deep
    pipeline and a forced drain, with the probe on for one batch; bit-exact.
    wgs > 0 shrinks the K3 grid to that many workgroups (HBX_K3_WGS), so each
    MD5 wave and its producer walk many groups in one launch.  q2/q4: K3Q,
    each slice in 2 / 4 items handed out through the launch's queue (a
    chain's slice continues on another wave, possibly another CU).  plan_cut: at
    join lag 2 (2: at any lag >= 2) the next launch is planned ahead on the cut
    stream (mode 3)."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K3_PROD", "0" if prod == "0" else "1")
    monkeypatch.setenv("HBX_K3_PSETS", "3" if prod == "p3" else "2")  # p3: three producer register sets
    monkeypatch.setenv("HBX_K3_ITEMS", prod[1:] if prod.startswith("q") else "0")
    monkeypatch.setenv("HBX_PLAN_CUT", plan_cut)
    if wgs:
        monkeypatch.setenv("HBX_K3_WGS", str(wgs))
    batches = _device_batches(oracle, 3, 71 + md5_slice % 5)
    got, order = [], []
    with Engine(0, md5_slice=md5_slice, join_lag=join_lag) as e:
        k = e.knobs()
        assert k["k3_prod"] == (prod != "0") and (not wgs or k["md5_wgs"] == wgs)
        assert k["k3_items"] == (int(prod[1:]) if prod.startswith("q") else 0)
        assert k["k3_psets"] == (3 if prod == "p3" else 2)
        cut = (plan_cut == "1" and join_lag == 2) or (plan_cut == "2" and join_lag >= 2)
        assert k["plan_mode"] == (3 if cut else {1: 0, 2: 1}.get(join_lag, 2)), k
        for i in [0, 1, 2, 0, 2, 1, 1, 0, 2, 2, 0, 1]:
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
            order.append(i)
            if e.pending() >= 6:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
        e.set_k3_probe(True)
        for i in (1, 2):
            e.submit_device(batches[i][0].data_ptr(), batches[i][1], batches[i][2])
            order.append(i)
        got += [e.wait(), e.wait()]
        w = e.k3_wave_times()
        assert (w[:, 2] >= w[:, 0]).all()
        e.set_k3_probe(False)
    assert len(got) == len(order)
    for i, g in zip(order, got):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("prod", ["1", "p3", "s", "a"])
@pytest.mark.parametrize("md5_slice,join_lag", [(9, 1), (9, 2), (16384, 1), (0, 2)])
def test_k3_lane_path_groups_between_cooperative_ones(oracle, monkeypatch, md5_slice, join_lag, prod):
    """Advisor r05 (high): with a producer wave per MD5 wave, a group on the
    lane path (fewer than 8 blocks for some lane) is hashed without waiting
    for the producer, and the MD5 wave rewrites its chains' `next`.  Both
    waves must still agree on every group's count, so the producer derives it
    from the order entry (immutable during the launch), never from the chain
    table.  Here most groups are on the lane path and sit between cooperative
    ones in each wave's walk: thousands of tiny files (0-2 full blocks) and
    files of 8-15 full blocks in one bin (at slice 16,384 the last bin spans
    counts 0-15), blocks of 64 of each so that one wave of a 1-workgroup grid
    (HBX_K3_WGS=1, four MD5 waves) walks lane, lane, cooperative, ..; plus a
    few long files; bit-exact over several pipelined batches."""
    import torch
    from hashbox_amd import Engine, pack_arena_layout
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K3_PROD", "1")
    monkeypatch.setenv("HBX_K3_PSETS", "3" if prod == "p3" else "2")
    monkeypatch.setenv("HBX_K3_ITEMS", "0")
    monkeypatch.setenv("HBX_K3_WGS", "1")
    monkeypatch.setenv("HBX_K3_SPIN", "1" if prod == "s" else "0")  # s: stage waits without s_sleep
    monkeypatch.setenv("HBX_PLAN_ADDR", "0" if prod == "a" else "512")  # a: by count only (round-5 order)
    rng = np.random.default_rng(977 + md5_slice % 13)
    batches = []
    for b in range(3):
        sizes = []
        for blk in range(36):
            lo, hi = [(0, 120), (0, 120), (504, 1016)][(blk + b) % 3]
            sizes += [int(v) for v in rng.integers(lo, hi, 64)]
        sizes += [3 * MIN + 5, MAXB + 123, 40_000]
        files = [oracle.random_bytes(n, 5000 + 7919 * b + i) for i, n in enumerate(sizes)]
        offs, total = pack_arena_layout(sizes)
        host = np.zeros(total, np.uint8)
        for o, f in zip(offs, files):
            host[int(o):int(o) + f.size] = f
        batches.append((torch.from_numpy(host).to("cuda:0"), offs, sizes,
                        [oracle.store_file(f, fast=True) for f in files]))
    torch.cuda.synchronize()
    got, order = [], []
    with Engine(0, md5_slice=md5_slice, join_lag=join_lag) as e:
        k = e.knobs()
        assert k["k3_prod"] and k["md5_wgs"] == 1 and k["k3_spin"] == (prod == "s")
        assert k["plan_addr"] == (0 if prod == "a" else 512)
        for i in [0, 1, 2, 1, 0, 2]:
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
            order.append(i)
            if e.pending() >= 4:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
    for i, g in zip(order, got):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("join_lag,plan_addr", [(1, 512), (2, 512), (3, 512), (4, 512), (2, 0), (1, 7)])
def test_pipelined_steady_state(oracle, monkeypatch, join_lag, plan_addr):
    """A deep pipeline as bench.py drives it: submit, and wait only once
    `depth` batches are pending, so batches complete through the slice
    schedule rather than a forced drain.  Join lags 1-4: the plan inline on
    the scan stream (lag 1), on the hash stream (lag 2), one launch ahead on
    the scan stream (lag >= 3)."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_PLAN_ADDR", str(plan_addr))  # full slices ordered by data address (plan_bin)
    batches = _device_batches(oracle, 3, 57)
    got = []
    with Engine(0, md5_slice=4096, join_lag=join_lag) as e:  # 256 KiB per chain per launch: 32 per 8 MiB
        assert e.knobs()["plan_addr"] == plan_addr
        order = [i % 3 for i in range(40)]
        for i in order:
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
            if e.pending() >= 32 + join_lag + 1:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
        with pytest.raises(Exception):  # the lag is fixed while batches are pending
            e.submit_device(batches[0][0].data_ptr(), batches[0][1], batches[0][2])
            e.set_join_lag(1)
        got.append(e.wait())
        order.append(0)
    assert len(got) == len(order)
    for i, g in zip(order, got):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("period,md5_slice,join_lag,plan_cut,meta", [
    (2, 16384, 1, "1", "1"), (3, 16384, 2, "1", "1"), (4, 8192, 2, "0", "0"), (3, 4096, 3, "1", "1"),
    (4, 8192, 3, "2", "1"), (8, 9, 2, "1", "1"), (5, 3, 1, "1", "0"), (4, 0, 2, "1", "1"), (1, 4096, 3, "2", "1"),
    (4, 8192, 2, "1", "2"), (2, 64, 1, "0", "2")])
def test_k3_period(oracle, monkeypatch, period, md5_slice, join_lag, plan_cut, meta):
    """K3 period (hbx_set_k3_period): one K3 launch every `period` submits
    with period x the slice per chain, several batches joining one plan (the
    planner's fresh-list set), in a deep pipeline as bench.py drives it, then
    a forced drain with batches still unjoined, then a refilled arena ring
    (hbx_input_after_oldest).  Every batch bit-exact; the launch count follows
    the period; the period is fixed while batches are pending.  plan_cut 2:
    the preplan on the cut stream at lag 3 too; meta 0: the batch meta by
    SDMA copy instead of hbx_meta_fetch; meta 1: the meta copy inside the
    K1 gate kernel (hbx_k1_gate_meta, the default); meta 2: hbx_meta_fetch and
    the gate as two kernels."""
    import torch
    from hashbox_amd import Engine, HbxError
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_PLAN_CUT", plan_cut)
    monkeypatch.setenv("HBX_META_KERNEL", "0" if meta == "0" else "1")
    monkeypatch.setenv("HBX_GATE_META", "1" if meta == "1" else "0")
    batches = _device_batches(oracle, 3, 83 + period)
    got, order = [], []
    with Engine(0, md5_slice=md5_slice, join_lag=join_lag, k3_period=period) as e:
        k = e.knobs()
        assert k["k3_period"] == period and k["meta_kernel"] == (meta != "0") and k["plan_cut"] == int(plan_cut)
        assert k["gate_meta"] == (meta == "1")
        e.stage_totals(reset=True)
        nfull = ((8 << 20) + 8) >> 6
        lb = md5_slice * period if md5_slice else nfull
        depth = -(-nfull // lb) * period + join_lag + period
        n_sub = 6 * period + 3
        for j in range(n_sub):
            i = j % 3
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
            order.append(i)
            if e.pending() >= depth:
                got.append(e.wait())
        _, n = e.stage_totals()  # launches harvested so far <= launches issued: one per period
        assert n[3] <= -(-n_sub // period) + 1, (n, period)
        while e.pending():  # forced drains, batches unjoined
            got.append(e.wait())
        _, n = e.stage_totals()
        assert n[0] == n_sub
        with pytest.raises(HbxError):
            e.submit_device(batches[0][0].data_ptr(), batches[0][1], batches[0][2])
            order.append(0)
            e.set_k3_period(1)
        while e.pending():
            got.append(e.wait())
        # a ring of 2 arenas refilled with the batches' data while pending
        big = max(b[0].numel() for b in batches)
        ring = [torch.empty(big, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
        torch.cuda.synchronize()
        for j in range(4 * period):
            i = j % 3
            if e.pending() >= 2:
                e.input_after_oldest()
                e.input_fence(torch.cuda.current_stream().cuda_stream)
            ring[j % 2][:batches[i][0].numel()].copy_(batches[i][0])
            e.submit_device(ring[j % 2].data_ptr(), batches[i][1], batches[i][2])
            order.append(i)
            if e.pending() >= 2:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
    assert len(got) == len(order)
    for i, g in zip(order, got):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("lean", ["1", "0"])
def test_plan_stream_changes_in_one_context(oracle, monkeypatch, lean):
    """One context through join lags 1 -> 2 -> 3 -> 1: the plan moves from
    the scan stream (mode 0) to the hash stream (mode 1) to a preplan on the
    scan stream (mode 2) and back.  With lean marks (hbx_engine.hip) the plan
    bins are zeroed after each plan on the plan's stream, so every move must
    order the new stream after the old one's fill; the stage totals still count
    one K1, K2 and plan per batch.  HBX_LEAN_MARKS=0 runs the old schedule."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_LEAN_MARKS", lean)
    batches = _device_batches(oracle, 2, 61)
    with Engine(0, md5_slice=4096) as e:
        assert e.knobs()["lean_marks"] == int(lean)
        e.stage_totals(reset=True)
        n_batches = 0
        for lag in (1, 2, 3, 1):
            e.set_join_lag(lag)
            got, order = [], [i % 2 for i in range(6)]
            for i in order:
                dev, offs, sizes, _ = batches[i]
                e.submit_device(dev.data_ptr(), offs, sizes)
                if e.pending() >= 3:
                    got.append(e.wait())
            while e.pending():
                got.append(e.wait())
            n_batches += len(order)
            assert len(got) == len(order)
            for i, g in zip(order, got):
                for a, r in zip(g, batches[i][3]):
                    _check(a, r)
        ms, n = e.stage_totals()
        assert n[0] == n_batches and n[1] == n_batches and n[2] >= n_batches
        assert all(m > 0 for m in ms[:4])


def test_reserved_pipeline(oracle):
    """hbx_reserve pre-sizes the pool, chain tables and summaries; a pipeline
    that runs its scan stream two steps ahead stays bit-exact."""
    from hashbox_amd import Engine
    batches = _device_batches(oracle, 2, 43)
    got, order = [], [i % 2 for i in range(12)]
    with Engine(0, md5_slice=2048) as e:
        e.reserve(10, max(len(b[2]) for b in batches), max(int(sum(b[2])) for b in batches))
        for i in order:
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
            if e.pending() >= 8:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
        with pytest.raises(Exception):  # reserve is refused while batches are pending
            e.submit_device(batches[0][0].data_ptr(), batches[0][1], batches[0][2])
            e.reserve(2, 1, 1)
        got_last = e.wait()
    for i, g in zip(order + [0], got + [got_last]):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("scan,hash_", [("off", ""), ("0:64:2", ""), ("0:4096", "0:128"), ("prio:lo", "prio:hi")])
def test_stream_cu_sets(oracle, monkeypatch, scan, hash_):
    """Streams created on CU subsets or priorities (HBX_SCAN_CUS / HBX_HASH_CUS,
    A/B switches; the scan stream is masked to every CU by default) change
    only the schedule: the pipeline stays bit-exact."""
    from hashbox_amd import Engine
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_SCAN_CUS", scan)
    if hash_:
        monkeypatch.setenv("HBX_AB", "1")
        monkeypatch.setenv("HBX_HASH_CUS", hash_)
    batches = _device_batches(oracle, 2, 47)
    got, order = [], [0, 1, 0, 1]
    with Engine(0, md5_slice=1024) as e:
        for i in order:
            dev, offs, sizes, _ = batches[i]
            e.submit_device(dev.data_ptr(), offs, sizes)
        while e.pending():
            got.append(e.wait())
    for i, g in zip(order, got):
        for a, r in zip(g, batches[i][3]):
            _check(a, r)


@pytest.mark.parametrize("md5_slice", [65536, 4096])
def test_input_after_oldest_ring(oracle, md5_slice):
    """A ring of 3 device arenas refilled with NEW data while earlier batches
    are still pending: hbx_input_after_oldest orders each refill (an H2D copy
    on the engine's input stream) and the batch after the oldest pending
    batch's last MD5 launch, on the GPU.  With slice 65536 that launch was
    issued already (no drain); with 4096 it was not (the call drains).
    Every batch must match the oracle on ITS data, never the data that
    replaced it."""
    import ctypes
    import torch
    from hashbox_amd import Engine, _lib, pack_arena_layout
    L = _lib.load()
    rng = np.random.default_rng(71)
    sizes = [9 * MAXB + 5, 3 * MIN + 7, 2 * MAXB + 99]
    offs, total = pack_arena_layout(sizes)
    datas = []
    for j in range(6):
        host = np.zeros(total, np.uint8)
        for k, (o, n) in enumerate(zip(offs, sizes)):
            host[int(o):int(o) + n] = rng.integers(0, 256, n, dtype=np.uint8)
        datas.append(host)
    refs = [[oracle.store_file(h[int(o):int(o) + n], fast=True) for o, n in zip(offs, sizes)] for h in datas]
    pin = ctypes.c_void_p()
    assert L.hbx_alloc_pinned(total * 6, ctypes.byref(pin)) == 0
    staged = np.ctypeslib.as_array((ctypes.c_uint8 * (total * 6)).from_address(pin.value))
    for j, h in enumerate(datas):
        staged[j * total:(j + 1) * total] = h
    ring = [torch.empty(total, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
    torch.cuda.synchronize()
    got, order = [], []
    with Engine(0, md5_slice=md5_slice) as e:
        for j in range(12):
            if e.pending() >= 3:
                e.input_after_oldest()
            d = j % 6
            e.memcpy_h2d_async(ring[j % 3].data_ptr(), pin.value + d * total, total)
            e.submit_device(ring[j % 3].data_ptr(), offs, sizes)
            order.append(d)
            if e.pending() > 3:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
    L.hbx_free_pinned(pin)
    assert len(got) == 12
    for d, res in zip(order, got):
        for g, r in zip(res, refs[d]):
            _check(g, r)


def test_input_fence_orders_caller_stream(oracle):
    """The ring of test_input_after_oldest_ring refilled by the CALLER's own
    work (a device-to-device copy on a torch stream of its own) instead of
    hbx_memcpy_h2d_async: hbx_input_fence(ctx, stream) puts the wait for the
    launch that finishes the oldest batch on that stream, so the refill never
    overwrites bytes K3 is still hashing.  Every batch must match the oracle
    on ITS data."""
    import torch
    from hashbox_amd import Engine, pack_arena_layout
    rng = np.random.default_rng(73)
    sizes = [9 * MAXB + 5, 3 * MIN + 7, 2 * MAXB + 99]
    offs, total = pack_arena_layout(sizes)
    datas = []
    for j in range(4):
        host = np.zeros(total, np.uint8)
        for o, n in zip(offs, sizes):
            host[int(o):int(o) + n] = rng.integers(0, 256, n, dtype=np.uint8)
        datas.append(host)
    refs = [[oracle.store_file(h[int(o):int(o) + n], fast=True) for o, n in zip(offs, sizes)] for h in datas]
    src = [torch.from_numpy(h).to("cuda:0") for h in datas]
    ring = [torch.empty(total, dtype=torch.uint8, device="cuda:0") for _ in range(3)]
    side = torch.cuda.Stream(device=0)
    torch.cuda.synchronize()
    got, order = [], []
    with Engine(0, md5_slice=4096) as e:
        for j in range(10):
            if e.pending() >= 3:
                e.input_after_oldest()
                e.input_fence(side.cuda_stream)
            d = j % 4
            with torch.cuda.stream(side):
                ring[j % 3].copy_(src[d])
                e.submit_device(ring[j % 3].data_ptr(), offs, sizes)  # ordered after `side` (hbx_after_stream)
            order.append(d)
            if e.pending() > 3:
                got.append(e.wait())
        while e.pending():
            got.append(e.wait())
    assert len(got) == 10
    for d, res in zip(order, got):
        for g, r in zip(res, refs[d]):
            _check(g, r)

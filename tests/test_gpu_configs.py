"""GPU: every BASELINE config that is a parity case, at its stated size,
bit-exact against the oracle's literal storeFile loop (store.go:111-196) plus
block.go:96-111 framing.

* configs[0]: one 1 GiB uniform random file (PCG64 seed 1) — from disk through
  hbx_store_paths and hbx_store_paths_z (every chunk's zlib stream strictly
  inflated back to the chunk), from host memory through hbx_chunk_hash, and
  device-resident through the pipelined submit/wait path.
* configs[3]: the 32 GiB Zipf-duplicated corpus (256 x 128 MiB, ~50 % repeat
  content) through the synchronous device call and the pipelined time-sliced
  path (4 batches of 64 files in flight), every file against the oracle on
  all host cores.
* one file past 2^32 bytes (4 GiB + 1 MiB + 12,345): device-resident
  (synchronous and pipelined) and from disk.
* configs[4] at its stated size: 100,000 files of log-uniform 4 KiB-4 MiB
  sizes (seed 5, ~61 GB), a quarter of them compressible text, on /dev/shm,
  through hbx_store_paths and hbx_store_paths_zcb: every file of both calls
  checked against the oracle run over all 100,000 files on every host core
  (store.go:254-397 stores every file), the compressed streams of every tenth
  file (10,000 files) inflated strictly (zlib, Adler-32, no trailing bytes)
  and equal to their chunks, callbacks FIFO and each file reported once.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GIB = 1 << 30


def _threads():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return min(16, os.cpu_count() or 1)


@pytest.fixture
def big_tmp(tmp_path):
    """A scratch directory for GiBs of files: /dev/shm when present (the box's
    /tmp may be small), else pytest's tmp_path.  Removed afterwards."""
    import shutil
    import tempfile
    d = tempfile.mkdtemp(prefix="hbx_cfg_", dir="/dev/shm") if os.path.isdir("/dev/shm") else str(tmp_path)
    try:
        yield d
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _same(g, r):
    assert np.array_equal(g.cut_ends, r.cut_ends), "cut ends differ"
    assert np.array_equal(g.ids, r.ids), "block ids differ"


def _chunks(data, cut_ends):
    s = 0
    for e in cut_ends:
        yield data[s:int(e)]
        s = int(e)


def _check_streams(pairs, threads):
    """pairs: [(data, FileChunks with zstreams)]; every chunk's stream must
    inflate strictly to the chunk's bytes."""
    from oracle import deflate as Z
    from concurrent.futures import ThreadPoolExecutor
    work = []
    for data, res in pairs:
        pieces = list(_chunks(data, res.cut_ends))
        assert len(res.zstreams) == len(pieces)
        work.extend(zip(res.zstreams, pieces))

    def one(zp):
        return Z.inflate_strict(bytes(zp[0])) == zp[1].tobytes()

    with ThreadPoolExecutor(threads) as ex:
        ok = list(ex.map(one, work))
    assert all(ok), f"{ok.count(False)} zlib streams do not inflate to their chunks"


def test_configs0_one_gib_file(engine, oracle, big_tmp):
    import torch
    n = 1 << 30
    data = np.random.Generator(np.random.PCG64(1)).integers(0, 256, n, dtype=np.uint8)
    ref = oracle.store_file(data)
    assert ref.n_chunks > 100
    # host memory, one call (hbx_chunk_hash)
    got = engine.chunk_hash(data)
    _same(got, ref)
    assert got.content_type == ref.content_type == 3 and got.content_id == ref.content_id
    # from disk (hbx_store_paths), then with every chunk compressed (hbx_store_paths_z)
    p = os.path.join(big_tmp, "config0.bin")
    data.tofile(p)
    for compress in (False, True):
        (r,) = engine.store_paths([p], compress=compress)
        _same(r, ref)
        assert r.content_id == ref.content_id
        if compress:
            _check_streams([(data, r)], _threads())
    os.unlink(p)
    # device-resident, pipelined (hbx_submit_device / hbx_wait, time-sliced K3)
    from hashbox_amd import Engine
    d = torch.empty(n + 65536, dtype=torch.uint8, device="cuda:0")
    d[:n].copy_(torch.from_numpy(data))
    torch.cuda.synchronize()
    with Engine(0, md5_slice=4096) as e:
        e.submit_device(d.data_ptr(), [0], [n])
        (r,) = e.wait()
    _same(r, ref)
    assert r.content_id == ref.content_id
    del d
    torch.cuda.empty_cache()


def test_one_file_past_4_gib(engine, oracle, big_tmp):
    """A single file longer than 2^32 bytes (odd length): 64-bit positions in
    K1's tiles, K2's chain walk, the chains and the file reader, device-resident
    (synchronous and pipelined) and from disk, against the oracle."""
    import torch
    from hashbox_amd import Engine
    n = (4 << 30) + (1 << 20) + 12345
    d = torch.empty(n + 65536, dtype=torch.uint8, device="cuda:0")
    g = torch.Generator(device="cuda:0")
    g.manual_seed(44)
    d[:n].random_(0, 256, generator=g)
    data = d[:n].cpu().numpy()
    ref = oracle.store_file(data)
    assert ref.n_chunks > 400 and int(ref.cut_ends[-1]) == n
    (sync,) = engine.chunk_hash_device(d.data_ptr(), [0], [n])
    _same(sync, ref)
    with Engine(0, md5_slice=8192) as e:
        e.submit_device(d.data_ptr(), [0], [n])
        (pipe,) = e.wait()
    _same(pipe, ref)
    assert sync.content_id == pipe.content_id == ref.content_id and sync.content_type == 3
    del d
    torch.cuda.empty_cache()
    p = os.path.join(big_tmp, "past4g.bin")
    data.tofile(p)
    (r,) = engine.store_paths([p])
    os.unlink(p)
    _same(r, ref)
    assert r.content_id == ref.content_id


def test_configs3_zipf_32_gib(oracle):
    import torch
    import workloads as W
    from hashbox_amd import Engine
    files, fbytes = 256, 128 << 20
    total = files * fbytes
    arena = torch.empty(total + 65536, dtype=torch.uint8, device="cuda:0")
    rep = W.zipf_fill([arena], total, seed=4)
    assert 0.4 < rep < 0.6, rep
    offs = np.arange(files, dtype=np.uint64) * np.uint64(fbytes)
    lens = [fbytes] * files
    with Engine(0) as e:  # synchronous: one call over all 256 files
        sync = e.chunk_hash_device(arena.data_ptr(), offs, lens)
    with Engine(0, md5_slice=2048) as e:  # pipelined: 4 batches of 64 in flight
        for b0 in range(0, files, 64):
            e.submit_device(arena.data_ptr(), offs[b0:b0 + 64], lens[b0:b0 + 64])
        pipe = []
        while e.pending():
            pipe.extend(e.wait())
    host = arena[:total].cpu().numpy()
    del arena
    torch.cuda.empty_cache()
    refs = oracle.store_batch_mt([host[i * fbytes:(i + 1) * fbytes] for i in range(files)], _threads())
    assert len(sync) == len(pipe) == files
    chunks = 0
    for s, p, r in zip(sync, pipe, refs):
        _same(s, r)
        _same(p, r)
        assert s.content_id == p.content_id and s.content_type == p.content_type
        assert s.content_type == (3 if r.n_chunks > 1 else 2)
        chunks += r.n_chunks
    assert chunks > 5000


def _text_pool(g, n):
    words = [bytes(g.integers(97, 123, int(k), dtype=np.uint8)) for k in g.integers(2, 10, 4096)]
    ranks = np.minimum(g.zipf(1.2, n // 4), len(words)) - 1
    return np.frombuffer(b" ".join(words[int(r)] for r in ranks), np.uint8)[:n]


def test_configs4_hundred_thousand_files_on_disk(engine, oracle, big_tmp):
    from concurrent.futures import ThreadPoolExecutor
    g = np.random.Generator(np.random.PCG64(5))
    n = 100_000
    sizes = np.exp(g.uniform(np.log(4096), np.log(4 << 20), n)).astype(np.int64)
    rand = g.integers(0, 256, 256 << 20, dtype=np.uint8)
    text = _text_pool(g, 16 << 20)
    offs = g.integers(0, 1 << 40, n)
    datas, paths = [], []
    for i in range(n):  # every file a view into one of two pools: no second copy in host memory
        pool = text if i % 4 == 0 else rand
        o = int(offs[i]) % (pool.size - int(sizes[i]))
        datas.append(pool[o:o + int(sizes[i])])
        paths.append(os.path.join(big_tmp, f"{i // 1000:03d}_{i:06d}.bin"))
    threads = _threads()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: datas[i].tofile(paths[i]), range(n)))
    total = int(sizes.sum())
    assert total > 50e9, total  # BASELINE configs[4]: 100 k files, 4 KiB-4 MiB
    refs = oracle.store_batch_mt(datas, threads)
    plain = engine.store_paths(paths, sizes=sizes, batch_bytes=1 << 30)
    # the content id (store.go:187-196): the one chunk's id, else the chain
    # block's id over the chunk ids (oracle chain_id, hashback.go:156-170)
    cids = [r.ids[0].tobytes() if r.n_chunks == 1 else oracle.chain_id(r.ids) for r in refs]
    for r, a, cid in zip(refs, plain, cids):
        _same(a, r)
        assert a.content_type == (2 if r.n_chunks == 1 else 3) and a.content_id == cid
    del plain
    seen = []

    def on_batch(first, count):
        seen.append((first, count))

    comp = engine.store_paths(paths, sizes=sizes, compress=True, on_batch=on_batch, batch_bytes=1 << 30)
    # the callbacks cover every file once, in order
    nxt = 0
    for first, count in seen:
        assert first == nxt and count > 0
        nxt += count
    assert nxt == n and len(seen) > 4
    single = 0
    for r, b, cid in zip(refs, comp, cids):
        _same(b, r)
        assert b.content_id == cid and b.content_type == (2 if r.n_chunks == 1 else 3)
        assert len(b.zstreams) == r.n_chunks
        single += r.n_chunks == 1
    assert 0 < single < n
    # the streams of every tenth file: strict inflate back to its chunks;
    # text compresses
    zin = zout = 0
    for i in range(0, n, 5000):
        _check_streams([(datas[j], comp[j]) for j in range(i, min(n, i + 5000), 10)], threads)
    for i in range(0, n, 4):
        zin += datas[i].size
        zout += sum(int(z.size) for z in comp[i].zstreams)
    assert zout < 0.6 * zin, (zout, zin)

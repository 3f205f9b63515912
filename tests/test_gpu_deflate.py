"""GPU: zlib block compression on the device (hbx_deflate_blocks*, kernels
K7a/K7s/K7b; HashboxBlock.CompressData, pkg/core/block.go:133-184).

Parity bar for this path (the output need not be bit-identical,
the server inflates and re-hashes, block.go:159-166): every stream must be a
complete RFC 1950 stream that inflates to exactly the block's data with a
correct Adler-32 (checked by CPython's zlib, oracle/deflate.py), within
hbx_deflate_bound.  Compression must also be real on compressible data.
"""
import numpy as np
import pytest

from oracle import deflate as OD

pytestmark = pytest.mark.gpu


def _text(n, seed):
    rng = np.random.default_rng(seed)
    words = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 10, 400)]
    out = bytearray()
    while len(out) < n:
        out += words[int(rng.zipf(1.3)) % len(words)] + b" "
    return bytes(out[:n])


def _check(engine, blocks):
    outs = engine.deflate_blocks(blocks)
    assert len(outs) == len(blocks)
    for b, z in zip(blocks, outs):
        assert z[:2] == b"\x78\x9c"
        assert len(z) <= engine.deflate_bound(len(b))
        assert OD.inflate_strict(z) == bytes(b)
    return outs


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 127, 128, 129, 1000, 32767, 32768, 32769, 65536, 100_001])
def test_edge_lengths_random_text_zero(engine, n):
    rng = np.random.default_rng(n)
    _check(engine, [rng.integers(0, 256, n, dtype=np.uint8).tobytes(), _text(n, n), bytes(n), b"ab" * (n // 2)])


def test_random_is_stored_and_text_compresses(engine):
    rng = np.random.default_rng(1)
    rnd = rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    txt = _text(3 << 20, 2)
    zr, zt, zz = _check(engine, [rnd, txt, bytes(1 << 20)])
    assert len(zr) == len(rnd) + 5 * (len(rnd) // 32768) + 11  # all stored: +5 B per 32 KiB segment
    ref = len(OD.compress_ref(txt))
    assert len(zt) < 0.75 * len(txt), (len(zt), len(txt))
    assert len(zt) < 1.4 * ref, (len(zt), ref)  # per-segment dynamic Huffman, 32 KiB windows vs zlib -6
    assert len(zz) < (1 << 20) // 16  # >= one match token per 64-byte parse range


def test_mixed_batch(engine):
    rng = np.random.default_rng(7)
    blocks = []
    for i in range(400):
        n = int(rng.choice([0, 1, 17, 4096, 16384, 40000, 70000, 200000]))
        kind = i % 4
        if kind == 0:
            blocks.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        elif kind == 1:
            blocks.append(_text(n, i))
        elif kind == 2:
            blocks.append(bytes([i & 255]) * n)
        else:
            per = rng.integers(0, 256, 37, dtype=np.uint8).tobytes()
            blocks.append((per * (n // 37 + 1))[:n])
    _check(engine, blocks)


def test_device_odd_offsets(engine):
    import torch
    rng = np.random.default_rng(9)
    datas = [_text(50_000, 1), rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes(), bytes(33_333), b"x"]
    offs, pos = [], 3
    for d in datas:  # inputs at odd byte offsets, as chunks inside a file are
        offs.append(pos)
        pos += len(d) + 7
    host = np.zeros(pos + 64, np.uint8)
    for o, d in zip(offs, datas):
        host[o:o + len(d)] = np.frombuffer(d, np.uint8)
    src = torch.from_numpy(host).to("cuda:0")
    caps = [engine.deflate_bound(len(d)) for d in datas]
    out_offs, q = [], 1
    for c in caps:  # outputs at odd offsets too
        out_offs.append(q)
        q += c + 5
    dst = torch.zeros(q + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    lens = engine.deflate_blocks_device(src.data_ptr(), offs, [len(d) for d in datas], dst.data_ptr(), out_offs, caps)
    out = dst.cpu().numpy()
    for d, o, k in zip(datas, out_offs, lens):
        assert OD.inflate_strict(out[o:o + int(k)].tobytes()) == d
    # nothing written outside the streams
    mask = np.ones(out.size, bool)
    for o, k in zip(out_offs, lens):
        mask[o:o + int(k)] = False
    assert not out[mask].any()


def test_capacity_refused(engine):
    import torch
    from hashbox_amd import HbxError
    src = torch.zeros(1024, dtype=torch.uint8, device="cuda:0")
    dst = torch.zeros(1024, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(HbxError):
        engine.deflate_blocks_device(src.data_ptr(), [0], [900], dst.data_ptr(), [0], [900])


def test_store_paths_compressed(engine, tmp_path):
    # the client's send path end to end: files on disk -> chunks + ids + one zlib stream per chunk
    rng = np.random.default_rng(12)
    paths, datas = [], []
    for i in range(44):  # > 64 MiB in total: several pipelined batches
        kind = i % 4
        n = int(rng.integers(1, 3 << 20)) if i % 11 else [0, 100, 131_073, 9 << 20][i // 11]
        d = (rng.integers(0, 256, n, dtype=np.uint8).tobytes() if kind == 0 else _text(n, i) if kind == 1
             else bytes(n) if kind == 2 else (rng.integers(0, 256, 5000, dtype=np.uint8).tobytes() * (n // 5000 + 1))[:n])
        p = tmp_path / f"f{i:02d}"
        p.write_bytes(d)
        paths.append(p)
        datas.append(d)
    plain = engine.store_paths(paths, io_threads=4)
    comp = engine.store_paths(paths, io_threads=4, compress=True)
    for d, a, b in zip(datas, plain, comp):
        assert np.array_equal(a.cut_ends, b.cut_ends) and np.array_equal(a.ids, b.ids)
        assert a.content_id == b.content_id
        assert len(b.zstreams) == b.n_chunks
        starts, ends = b.chunk_bounds()
        for s, e, z in zip(starts, ends, b.zstreams):
            assert OD.inflate_strict(z) == d[int(s):int(e)]


def test_store_paths_on_batch_covers_every_file_once(engine, tmp_path):
    """store_paths(compress=True, on_batch=...) -> hbx_store_paths_zcb: the
    per-batch callback reports every file exactly once, in order, and the
    streams it announced are the ones returned (SURVEY §8f3 send path)."""
    rng = np.random.default_rng(21)
    paths = []
    for i in range(112):  # ~224 MiB: four or more 64 MiB (the minimum) batches, so the
        # asynchronous compression stages are reused (drained before reuse)
        p = tmp_path / f"g{i:02d}"
        p.write_bytes(rng.integers(0, 256, int(rng.integers(1, 4 << 20)), dtype=np.uint8).tobytes())
        paths.append(p)
    seen = []
    res = engine.store_paths(paths, io_threads=4, batch_bytes=64 << 20, compress=True,
                             on_batch=lambda first, count: seen.append((first, count)))
    assert len(seen) >= 4
    assert [f for a, c in seen for f in range(a, a + c)] == list(range(len(paths)))
    for p, r in zip(paths, res):
        ref = engine.chunk_hash(np.fromfile(p, np.uint8))
        assert np.array_equal(r.ids, ref.ids)
        data = p.read_bytes()
        starts, ends = r.chunk_bounds()
        for j, (z, a, b) in enumerate(zip(r.zstreams, starts, ends)):
            if j < 2 or paths.index(p) % 8 == 0:  # every stream of every 8th file
                assert OD.inflate_strict(bytes(z)) == data[int(a):int(b)]


def test_store_paths_on_batch_needs_compress(engine, tmp_path):
    p = tmp_path / "x"
    p.write_bytes(b"abc")
    with pytest.raises(ValueError):
        engine.store_paths([p], on_batch=lambda a, c: None)


def test_entropy_early_out_boundaries(engine):
    """K7's incompressible early-out (order-0 entropy >= 7.97 bits per byte and
    no sampled 4-byte repeat in the window -> stored, no parse): plain random
    bytes are stored; random bytes that repeat within the window (periods of
    8 KiB and 20 KiB) are parsed and compress; bytes over
    200 symbols (7.64 bits) still get a Huffman code; a block below 4 KiB
    takes the full parse; mixes of both kinds in one block stay valid."""
    rng = np.random.default_rng(33)
    rnd = rng.integers(0, 256, 1 << 16, dtype=np.uint8).tobytes()            # 64 KiB random: stored
    rep = rng.integers(0, 256, 8192, dtype=np.uint8).tobytes() * 8         # 64 KiB, entropy ~8 bits, LZ-redundant
    rep20 = rng.integers(0, 256, 20480, dtype=np.uint8).tobytes() * 4      # 80 KiB, period 20 KiB
    few = rng.integers(0, 200, 1 << 17, dtype=np.uint8).tobytes()            # log2(200) = 7.64 bits
    small = rng.integers(0, 256, 1500, dtype=np.uint8).tobytes() * 2         # 3000 B: below the early-out
    mix = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes() + _text(60000, 5)
    zn, zr, z20, zf, zs, zm = _check(engine, [rnd, rep, rep20, few, small, mix])
    assert len(zn) == len(rnd) + 5 * (len(rnd) // 32768) + 11  # stored segments
    assert len(zr) < 0.25 * len(rep), (len(zr), len(rep))     # the parse found the repeats
    assert len(z20) < 0.6 * len(rep20), (len(z20), len(rep20))
    assert len(zf) < 0.98 * len(few), (len(zf), len(few))     # Huffman-coded, not stored
    assert len(zs) < 0.7 * len(small), (len(zs), len(small))  # the full parse matched the repeat
    assert len(zm) < len(mix), (len(zm), len(mix))            # the text half compresses


def test_parse_handoff_that_does_not_settle(engine):
    """K7's parse hands each thread's end on as the next thread's start for at
    most 8 rounds.  Zero runs never settle (the hand-off cycles with period 4);
    long matches of repeated phrases at shifting alignments make a re-parsed
    thread end past its successor's end.  The recording ranges must still tile
    the segment exactly (hbx_deflate.hip: a running maximum over the starts
    when the hand-off did not settle), else bytes are coded twice and the
    stream inflates to the wrong data.  Every block is strictly inflated."""
    rng = np.random.default_rng(4242)
    blocks = []
    for i in range(160):
        out = bytearray(bytes(1024 + 37 * i))  # a zero run of >= 1 KiB
        phrase = _text(int(rng.integers(259, 900)), 1000 + i)
        while len(out) < 70_000:
            kind = int(rng.integers(0, 4))
            if kind == 0:
                out += bytes(int(rng.integers(1, 3000)))
            elif kind == 1:
                out += phrase[int(rng.integers(0, 64)):]
            elif kind == 2:
                out += bytes(rng.integers(0, 256, int(rng.integers(1, 70)), dtype=np.uint8))
            else:
                out += (phrase[:int(rng.integers(4, 300))]) * int(rng.integers(1, 6))
        blocks.append(bytes(out[:int(rng.integers(40_000, 70_000))]))
    for k in (1, 2, 3, 5, 7, 63, 65, 257, 259):  # zeros with a single byte every k*64 + j bytes
        for j in (0, 1, 31):
            b = bytearray(65_536)
            b[j::64 * k + j + 1] = b"\x01" * len(b[j::64 * k + j + 1])
            blocks.append(bytes(b))
    _check(engine, blocks)


def test_history_reaches_back_32k(engine):
    """A segment's matches may reach the whole 32 KiB before it (round 4;
    16 KiB before): X Y X Y with 12 KiB of random letters each (order-0
    entropy 4.7 bits, so no segment is stored by the early-out) puts the
    second copies at distance 24 KiB, and the second segment ([32, 48) KiB)
    lies entirely inside them: with the history it costs almost nothing, an
    order-0 code alone would take ~9.4 KiB for it.  Then a copy at exactly the
    window's reach, distance 32,768.  Strict inflate checks every distance."""
    rng = np.random.default_rng(7)
    letters = lambda n: rng.integers(97, 123, n, dtype=np.uint8).tobytes()  # noqa: E731
    x, y = letters(12 << 10), letters(12 << 10)
    (z,) = _check(engine, [x + y + x + y])
    assert len(z) < 0.6 * (24 << 10) + 2048, len(z)  # X0 Y0 at order-0 cost, the copies nearly free (no history: >= 23 KiB)
    w = letters(32 << 10)
    (z2,) = _check(engine, [w + w[:16 << 10]])
    assert len(z2) < 0.6 * (32 << 10) + 2048, len(z2)  # (no history: >= 28 KiB)


def test_random_repeat_in_history_is_parsed(engine):
    """K7e samples a segment's history as well as the segment: random bytes
    whose only repeat lies in the 32 KiB before the segment are parsed (and
    matched there), not stored.  The first 32 KiB segment stays stored."""
    rng = np.random.default_rng(11)
    w = rng.integers(0, 256, 32 << 10, dtype=np.uint8).tobytes()
    (z,) = _check(engine, [w + w[:16 << 10]])
    assert len(z) < (32 << 10) + 1024, len(z)  # stored first segment + a nearly free second


def test_shared_code_groups(engine):
    """Round 4: kGroup = 4 consecutive parsed segments of a block share one
    dynamic code (K7h): one header, one end of block and sync flush, and each
    member's bits continue the previous member's mid-byte.  Edges: partial
    groups (2, 3, 5, 9 segments), a last member of a few bits (a 4-byte match
    at distance 4), a member of zeros (a few hundred bits), a stored random
    segment inside a group (no sharing there), a group piece past 64 KiB
    (7-bit random bytes), and a text block whose group pieces must each end
    in the only sync flush of the group."""
    seg = 32768
    t = _text(12 * seg, 3)
    rng = np.random.default_rng(5)
    rnd = rng.integers(0, 256, seg, dtype=np.uint8).tobytes()
    blocks = [t[:n] for n in (seg + 1, seg + 3, 2 * seg + 5, 3 * seg + 1, 4 * seg, 4 * seg + 3, 5 * seg + 17,
                              9 * seg + 100)]
    blocks.append(t[: seg - 4] + b"wxyz" + b"wxyz")  # second segment: one 4-byte match
    blocks.append(t[:seg] + bytes(seg) + t[seg : 3 * seg])  # zeros in the middle of a group
    blocks.append(t[:seg] + rnd + t[seg : 3 * seg])  # a stored member: the group codes alone
    blocks.append(rnd + t[: 3 * seg] + rnd + t[3 * seg : 6 * seg])
    blocks.append(rng.integers(0, 128, 4 * seg + 7, dtype=np.uint8).tobytes())  # 7 bits/B: a ~112 KiB group piece
    _check(engine, blocks)
    big = _text(4 << 20, 9)
    (z,) = _check(engine, [big])
    # 128 segments in 32 groups: one sync flush (00 00 FF FF) per group + the final block's
    assert z.count(b"\x00\x00\xff\xff") <= 128 // 4 + 2, z.count(b"\x00\x00\xff\xff")


def test_group_that_codes_alone(engine):
    """A group whose shared code loses (K7h's second pass): random segments
    that K7e still parses (each holds a repeated 256-byte run, so a sampled
    value repeats) code as stored, member by member; and a text member with
    such a random member, where the shared code may or may not win.  Both
    must inflate exactly and stay within the stored size."""
    seg = 32768
    rng = np.random.default_rng(23)

    def rnd_with_repeat():
        r = bytearray(rng.integers(0, 256, seg, dtype=np.uint8).tobytes())
        r[20000:20256] = r[1000:1256]
        return bytes(r)

    a, b, c = rnd_with_repeat(), rnd_with_repeat(), rnd_with_repeat()
    z1, z2, z3 = _check(engine, [a + b, a + b + c, _text(seg, 4) + b])
    assert len(z1) <= 2 * (seg + 5) + 11, len(z1)
    assert len(z2) <= 3 * (seg + 5) + 11, len(z2)

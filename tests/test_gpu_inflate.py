"""GPU: zlib inflate on the device (hbx_inflate_blocks_device, K8;
HashboxBlock.UncompressData, pkg/core/block.go:113-131), the read side
VerifyBlock needs for stored (compressed) blocks.  The streams come from
CPython's zlib at every level (stored, fixed and dynamic blocks, 32 KiB
windows; the stand-in for Go's compress/zlib) and from the device deflate
(K7); the inflated bytes must equal the originals exactly.  Corrupt streams
must fail with a status, never fault.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["wave", "lane", "split"])
def k8_mode(request, monkeypatch):
    """Every decoder: a wave per stream, a lane per stream (picked for tens
    of thousands of short compressible streams) and long streams split into
    regions decoded in parallel (hbx_inflate_split.hip; forced here for every
    stream of >= 2 regions, compressible or not)."""
    monkeypatch.setenv("HBX_AB", "1")
    monkeypatch.setenv("HBX_K8_MODE", request.param)
    return request.param


def _text(n, seed):
    rng = np.random.default_rng(seed)
    words = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 10, 300)]
    out = bytearray()
    while len(out) < n:
        out += words[int(rng.zipf(1.3)) % len(words)] + b" "
    return bytes(out[:n])


def _datas():
    rng = np.random.default_rng(3)
    out = []
    for n in (0, 1, 100, 32768, 40000, 300_000):
        out += [rng.integers(0, 256, n, dtype=np.uint8).tobytes(), _text(n, n), bytes(n),
                (rng.integers(0, 256, 33000, dtype=np.uint8).tobytes() * (n // 33000 + 1))[:n]]  # far matches
    return out


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_inflate_zlib_levels(engine, level):
    datas = _datas()
    streams = [zlib.compress(d, level) for d in datas]
    outs, st = engine.inflate_blocks(streams, [len(d) + 16 for d in datas])
    assert st.tolist() == [0] * len(datas)
    for d, o in zip(datas, outs):
        assert o == d


def test_inflate_device_deflate_and_big(engine):
    datas = [_text(3 << 20, 1), np.random.default_rng(2).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()]
    streams = engine.deflate_blocks(datas) + [zlib.compress(d, 6) for d in datas]
    outs, st = engine.inflate_blocks(streams, [3 << 20] * 4)
    assert st.tolist() == [0] * 4
    assert outs[0] == datas[0] and outs[1] == datas[1] and outs[2] == datas[0] and outs[3] == datas[1]


def test_inflate_corrupt_streams_fail_cleanly(engine):
    d = _text(50_000, 9)
    z = zlib.compress(d, 6)
    bad = [z[:len(z) // 2],                      # truncated
           z[:-1],                               # Adler cut
           z[:-4] + bytes(4),                    # wrong Adler
           b"\x78\x9d" + z[2:],                  # header check bits
           z[:10] + bytes([z[10] ^ 0xFF]) + z[11:],  # flipped bits inside the data
           b"",
           bytes(64)]
    outs, st = engine.inflate_blocks(bad + [z], [len(d)] * len(bad) + [len(d)])
    assert all(s != 0 for s in st[:len(bad)])
    assert st[-1] == 0 and outs[-1] == d
    # capacity one byte short
    _, st2 = engine.inflate_blocks([z], [len(d) - 1])
    assert st2.tolist() == [3]


def test_verify_compressed_blocks(engine, oracle):
    """VerifyBlock of zlib blocks (block.go:152-166): inflate on the device,
    then HashData of the result against the expected ids."""
    import torch
    rng = np.random.default_rng(11)
    datas = [_text(int(n), int(n)) for n in rng.integers(1, 200_000, 50)]
    links = [[rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(i % 3)] for i in range(50)]
    want = [oracle.block_id(np.frombuffer(d, np.uint8), l) for d, l in zip(datas, links)]
    streams = [zlib.compress(d, 6) for d in datas]
    outs, st = engine.inflate_blocks(streams, [len(d) + 64 for d in datas])
    assert st.tolist() == [0] * 50
    ids, ok, bad = engine.verify_blocks(outs, links, expect=want)
    assert bad == 0 and ok.all()


def _long_streams():
    """Long streams the split path must resolve or hand back: zlib at levels
    1/6/9, with periodic sync flushes (byte-aligned block starts), the device
    deflate's own streams (sync flush after every 32 KiB piece), a run of
    zeros (a region's symbols overflow its scratch), and half random / half
    text (stored and Huffman blocks in one stream)."""
    import zlib as Z
    rng = np.random.default_rng(21)
    datas, streams = [], []
    for i, n in enumerate([1 << 20, 3 << 20, (5 << 20) + 12345, 700_000]):
        d = _text(n, 100 + i)
        for level in (1, 6, 9):
            datas.append(d)
            streams.append(Z.compress(d, level))
        co = Z.compressobj(6)
        parts = [co.compress(d[k:k + 100_000]) + co.flush(Z.Z_SYNC_FLUSH) for k in range(0, len(d), 100_000)]
        datas.append(d)
        streams.append(b"".join(parts) + co.flush())
    z = bytes(4 << 20)
    mix = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() + _text(2 << 20, 7)
    for d in (z, mix):
        datas.append(d)
        streams.append(Z.compress(d, 6))
    return datas, streams


def test_inflate_long_streams(engine):
    datas, streams = _long_streams()
    k7 = [_text(4 << 20, 31), _text((2 << 20) + 777, 32)]
    datas += k7
    streams += engine.deflate_blocks(k7)
    outs, st = engine.inflate_blocks(streams, [len(d) for d in datas])
    assert st.tolist() == [0] * len(datas)
    for d, o in zip(datas, outs):
        assert o == d


def test_split_resolves_text_streams(engine, k8_mode):
    """The split path must decode long zlib -6 text streams itself (the
    engine's counters: every stream split, none handed back to the wave
    kernel), not merely fall back."""
    import zlib as Z
    if k8_mode != "split":
        pytest.skip("split mode only")
    datas = [_text((3 << 20) + 1000 * i, 200 + i) for i in range(6)]
    streams = [Z.compress(d, 6) for d in datas] + engine.deflate_blocks(datas[:2])
    datas = datas + datas[:2]
    k0 = engine.knobs()
    outs, st = engine.inflate_blocks(streams, [len(d) for d in datas])
    k1 = engine.knobs()
    assert st.tolist() == [0] * len(datas)
    assert all(o == d for d, o in zip(datas, outs))
    assert k1["k8_split_streams"] - k0["k8_split_streams"] == len(datas)
    assert k1["k8_split_fallbacks"] - k0["k8_split_fallbacks"] == 0, (k0, k1)


def test_inflate_corrupt_long_streams(engine):
    """Corrupt long streams fail with a status in every mode (the split path
    hands them to the wave kernel, whose status is the answer)."""
    import zlib as Z
    d = _text(2 << 20, 41)
    z = Z.compress(d, 6)
    rng = np.random.default_rng(5)
    bad = [z[:len(z) // 2], z[:-4] + bytes(4), z[:-1]]
    for at in rng.integers(100, len(z) - 100, 6):
        bad.append(z[:int(at)] + bytes([z[int(at)] ^ 0x5A]) + z[int(at) + 1:])
    outs, st = engine.inflate_blocks(bad + [z], [len(d)] * (len(bad) + 1))
    assert st[-1] == 0 and outs[-1] == d
    for b, s_, o in zip(bad, st[:-1], outs[:-1]):
        assert s_ != 0 or o == d, "a corrupt stream inflated to different data with status 0"
    assert all(s_ != 0 for s_ in st[:3])

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


@pytest.fixture(autouse=True, params=["wave", "lane"])
def k8_mode(request, monkeypatch):
    """Both decoders: a wave per stream (the default) and a lane per stream
    (picked for tens of thousands of short compressible streams)."""
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

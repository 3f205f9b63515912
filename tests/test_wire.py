"""CPU: the wire framing of the block-store exchange (hbx_wire_*; SURVEY
§8f3) against the oracle's restatement of ProtocolMessage.Serialize and
HashboxBlock.Serialize (oracle/wire.py; pkg/core/protocol.go:184-264,
pkg/core/block.go:56-69).  Pure host code: runs without a GPU."""
import ctypes
import random

import pytest

from oracle import wire as OW

_lib = pytest.importorskip("hashbox_amd._lib")


@pytest.fixture(scope="module")
def L():
    return _lib.load()


def _parse(L, buf):
    m = _lib.WireMsg()
    src = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
    rc = L.hbx_wire_parse(src, len(buf), ctypes.byref(m))
    return rc, m, src


@pytest.mark.parametrize("mtype", [OW.ALLOCATE, OW.READ, OW.ACKNOWLEDGE & OW.SERVER_MASK, OW.READ & OW.SERVER_MASK])
def test_id_messages(L, mtype):
    rng = random.Random(mtype)
    for num in (0, 1, 0xBEEF, 0xFFFF):
        bid = rng.randbytes(16)
        out = (ctypes.c_uint8 * 22)()
        assert L.hbx_wire_encode_id(num, mtype, bid, out) == 0
        assert bytes(out) == OW.id_msg(num, mtype, bid)
        rc, m, _ = _parse(L, bytes(out) + b"next")
        assert rc == 0 and m.num == num and m.type == mtype and bytes(m.id) == bid and m.total_len == 22


@pytest.mark.parametrize("nlinks,n", [(0, 0), (0, 1), (3, 1000), (0, 70000)])
def test_block_messages(L, nlinks, n):
    rng = random.Random(n)
    bid, links, data = rng.randbytes(16), [rng.randbytes(16) for _ in range(nlinks)], rng.randbytes(n)
    for mtype in (OW.WRITE, OW.WRITE & OW.SERVER_MASK):
        hdr = ctypes.create_string_buffer(64 + 16 * nlinks)
        used = ctypes.c_uint64()
        lk = b"".join(links) or None
        assert L.hbx_wire_encode_block_header(7, mtype, bid, lk, nlinks, OW.ZLIB, n, hdr, len(hdr.raw),
                                              ctypes.byref(used)) == 0
        wire = hdr.raw[:used.value] + data
        assert wire == OW.block_msg(7, mtype, bid, links, OW.ZLIB, data)
        rc, m, src = _parse(L, wire)
        assert rc == 0 and m.type == mtype and bytes(m.id) == bid and m.n_links == nlinks
        assert m.data_type == OW.ZLIB and m.data_len == n and m.total_len == len(wire)
        assert m.header_len == 31 + 16 * nlinks
        if n:
            assert ctypes.string_at(m.data, n) == data
        # every strict prefix is incomplete, never an error
        for cut in sorted({0, 1, 5, 6, 21, 22, 25, 26, m.header_len - 1, m.header_len, len(wire) - 1}):
            if 0 <= cut < len(wire):
                assert _parse(L, wire[:cut])[0] == -3


def test_other_messages_and_errors(L):
    rc, m, _ = _parse(L, OW.greeting(3, 1))
    assert rc == 0 and m.type == OW.GREETING and m.data_len == 1 and m.total_len == 10
    rc, m, _ = _parse(L, OW.error_msg(9, b"no such block"))
    assert rc == 0 and m.data_len == 13 and ctypes.string_at(m.data, 13) == b"no such block"
    rc, m, _ = _parse(L, OW.header(1, OW.GOODBYE))
    assert rc == 0 and m.total_len == 6
    assert _parse(L, OW.header(1, 0x12345678) + bytes(16))[0] == -7  # "invalid protocol message"
    out = (ctypes.c_uint8 * 22)()
    assert L.hbx_wire_encode_id(0, OW.WRITE, bytes(16), out) == -1  # not an id message

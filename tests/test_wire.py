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


# ---- pkg/core/protocol_test.go:71-285 (TestMessageSerialization), mirrored --
def _rand_msg_string(rng):  # randomMsgString: printable text of random length
    return bytes(rng.randrange(32, 127) for _ in range(rng.randrange(0, 200)))


def _rand_block(rng):  # randomHashboxBlock: raw data, one random link, id = HashData
    from oracle import oracle as O
    data, links = _rand_msg_string(rng), [rng.randbytes(16)]
    return {"BlockID": O.py_block_id(data, links), "Links": links, "DataType": OW.RAW, "Data": data}


def _rand_state(rng):
    return {"StateID": rng.randbytes(16), "BlockID": rng.randbytes(16), "Size": rng.randrange(1 << 63),
            "UniqueSize": rng.randrange(1 << 63)}


def _protocol_cases(rng):
    """Every (type, Data) TestMessageSerialization sends, in its order."""
    SM = OW.SERVER_MASK
    return [
        (OW.GREETING, {"Version": rng.randrange(1 << 32)}),
        (OW.GREETING & SM, {"SessionNonce": rng.randbytes(16)}),
        (OW.AUTHENTICATE, {"AccountNameH": rng.randbytes(16), "AuthenticationH": rng.randbytes(16)}),
        (OW.AUTHENTICATE & SM, None),
        (OW.GOODBYE, None),
        (OW.GOODBYE & SM, None),
        (OW.ERROR & SM, {"ErrorMessage": _rand_msg_string(rng)}),
        (OW.ALLOCATE, {"BlockID": rng.randbytes(16)}),
        (OW.ACKNOWLEDGE & SM, {"BlockID": rng.randbytes(16)}),
        (OW.READ & SM, {"BlockID": rng.randbytes(16)}),
        (OW.WRITE, {"Block": _rand_block(rng)}),
        (OW.READ, {"BlockID": rng.randbytes(16)}),
        (OW.WRITE & SM, {"Block": _rand_block(rng)}),
        (OW.ACCOUNT_INFO, {"AccountNameH": rng.randbytes(16)}),
        (OW.ACCOUNT_INFO & SM, {"DatasetList": [{"Name": _rand_msg_string(rng), "Size": rng.randrange(1 << 63),
                                                 "ListH": rng.randbytes(16)}]}),
        (OW.LIST_DATASET, {"AccountNameH": rng.randbytes(16), "DatasetName": _rand_msg_string(rng)}),
        (OW.LIST_DATASET & SM, {"States": [{"StateFlags": rng.randrange(256), "State": _rand_state(rng)}],
                                "ListH": rng.randbytes(16)}),
        (OW.ADD_DATASET_STATE, {"AccountNameH": rng.randbytes(16), "DatasetName": _rand_msg_string(rng),
                                "State": _rand_state(rng)}),
        (OW.ADD_DATASET_STATE & SM, None),
        (OW.REMOVE_DATASET_STATE, {"AccountNameH": rng.randbytes(16), "DatasetName": _rand_msg_string(rng),
                                   "StateID": rng.randbytes(16)}),
        (OW.REMOVE_DATASET_STATE & SM, None),
    ]


@pytest.mark.parametrize("seed", range(8))
def test_message_serialization(L, seed):
    """protocolPipeCompare for every message type: serialize, frame it with
    hbx_wire_parse (type, num, exact length; block fields for writ/WRIT),
    read it back, and compare — writ/WRIT by VerifyBlock (HashData of the
    parsed block equals its BlockID), the rest by deep equality."""
    from oracle import oracle as O
    rng = random.Random(1000 + seed)
    for mtype, data in _protocol_cases(rng):
        num = rng.randrange(1 << 16)
        wire = OW.serialize(num, mtype, data)
        rc, m, src = _parse(L, wire + b"\x00" * 7)  # trailing bytes of the next message
        assert rc == 0, hex(mtype)
        assert m.num == num and m.type == mtype and m.total_len == len(wire), hex(mtype)
        n2, t2, d2, used = OW.unserialize(wire)
        assert (n2, t2, used) == (num, mtype, len(wire))
        if mtype in (OW.WRITE, OW.WRITE & OW.SERVER_MASK):
            b = data["Block"]
            assert bytes(m.id) == b["BlockID"] and m.n_links == len(b["Links"]) and m.data_type == b["DataType"]
            assert m.data_len == len(b["Data"]) and ctypes.string_at(m.data, m.data_len) == b["Data"]
            assert ctypes.string_at(m.links, 16 * m.n_links) == b"".join(b["Links"])
            assert O.py_block_id(d2["Block"]["Data"], d2["Block"]["Links"]) == d2["Block"]["BlockID"]  # VerifyBlock
        else:
            assert d2 == data, hex(mtype)
            if mtype in (OW.ALLOCATE, OW.READ, OW.ACKNOWLEDGE & OW.SERVER_MASK, OW.READ & OW.SERVER_MASK):
                assert bytes(m.id) == data["BlockID"]
        # every strict prefix is incomplete, never an error or a wrong length
        for cut in range(len(wire)):
            assert _parse(L, wire[:cut])[0] == -3, (hex(mtype), cut)


def test_message_stream_framing(L):
    """A stream of every message type back to back frames message by message."""
    rng = random.Random(7)
    cases = _protocol_cases(rng) * 3
    stream = b"".join(OW.serialize(i, t, d) for i, (t, d) in enumerate(cases))
    pos, seen = 0, []
    while pos < len(stream):
        rc, m, _ = _parse(L, stream[pos:])
        assert rc == 0
        seen.append((m.num, m.type))
        pos += m.total_len
    assert pos == len(stream) and seen == [(i, t) for i, (t, _) in enumerate(cases)]
    # the old greeting "hola" has no data; an unknown type is refused
    assert _parse(L, OW.header(5, OW.OLD_GREETING))[1].total_len == 6
    assert _parse(L, OW.header(5, OW.ACCOUNT_INFO & 0x12345678))[0] == -7

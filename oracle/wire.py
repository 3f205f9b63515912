"""CPU restatement of the Hashbox wire protocol messages — TEST
INFRASTRUCTURE ONLY (tests/ and tools/ alone).

* ProtocolMessage.Serialize / Unserialize   pkg/core/protocol.go:184-264
  (u16 Num, u32 Type, then the Data struct's fields in declaration order;
  the type switch of Unserialize decides the struct)
* message types / server mask               pkg/core/protocol.go:37-70
* message structs                           pkg/core/protocol.go:72-174
* String, Dataset(Array), DatasetState,
  DatasetStateEntry/Array                   pkg/core/core.go:95-216
* HashboxBlock.Serialize                    pkg/core/block.go:56-69
* big-endian integers                       pkg/core/utils.go:73-88

Parity: pkg/core/protocol_test.go:71-285 exercises these messages as round
trips through the Go code itself (no byte fixtures), so the layouts are
pinned by source; tests/test_wire.py mirrors that test message by message.
"""
from __future__ import annotations

import struct
from typing import Optional, Sequence, Tuple

OLD_GREETING, GREETING, AUTHENTICATE, GOODBYE = 0x686F6C61, 0x68616C6F, 0x61757468, 0x71756974
ALLOCATE, READ, WRITE, ACKNOWLEDGE = 0x616C6C6F, 0x72656164, 0x77726974, 0x61636B6E
ACCOUNT_INFO, ADD_DATASET_STATE, LIST_DATASET, REMOVE_DATASET_STATE = 0x696E666F, 0x61646473, 0x6C697374, 0x64656C73
ERROR = 0x65727273
SERVER_MASK = 0xDFDFDFDF
RAW, ZLIB = 0xFF, 0x01
SM = SERVER_MASK

# Data struct of every type Unserialize knows (protocol.go:204-250): a list
# of (field, kind), or None for a message without Data.
SCHEMA = {
    GREETING: [("Version", "u32")],
    GREETING & SM: [("SessionNonce", "b128")],
    OLD_GREETING: None,
    AUTHENTICATE: [("AccountNameH", "b128"), ("AuthenticationH", "b128")],
    AUTHENTICATE & SM: None,
    GOODBYE: None,
    GOODBYE & SM: None,
    ERROR & SM: [("ErrorMessage", "str")],
    ALLOCATE: [("BlockID", "b128")],
    ACKNOWLEDGE & SM: [("BlockID", "b128")],
    READ & SM: [("BlockID", "b128")],
    WRITE: [("Block", "block")],
    READ: [("BlockID", "b128")],
    WRITE & SM: [("Block", "block")],
    ACCOUNT_INFO: [("AccountNameH", "b128")],
    ACCOUNT_INFO & SM: [("DatasetList", "datasets")],
    LIST_DATASET: [("AccountNameH", "b128"), ("DatasetName", "str")],
    LIST_DATASET & SM: [("States", "states"), ("ListH", "b128")],
    ADD_DATASET_STATE: [("AccountNameH", "b128"), ("DatasetName", "str"), ("State", "state")],
    ADD_DATASET_STATE & SM: None,
    REMOVE_DATASET_STATE: [("AccountNameH", "b128"), ("DatasetName", "str"), ("StateID", "b128")],
    REMOVE_DATASET_STATE & SM: None,
}


def header(num: int, mtype: int) -> bytes:
    return struct.pack(">HI", num, mtype)


def _state(s: dict) -> bytes:  # DatasetState.Serialize, core.go:163-169
    return s["StateID"] + s["BlockID"] + struct.pack(">qq", s["Size"], s["UniqueSize"])


def _field(kind: str, v) -> bytes:
    if kind == "u32":
        return struct.pack(">I", v)
    if kind == "b128":
        assert len(v) == 16
        return bytes(v)
    if kind == "str":  # String.Serialize, core.go:97-101
        return struct.pack(">I", len(v)) + bytes(v)
    if kind == "block":  # HashboxBlock.Serialize, block.go:56-69
        return (v["BlockID"] + struct.pack(">I", len(v["Links"])) + b"".join(v["Links"])
                + struct.pack(">BI", v["DataType"], len(v["Data"])) + v["Data"])
    if kind == "datasets":  # DatasetArray / Dataset.Serialize, core.go:118-139
        return struct.pack(">I", len(v)) + b"".join(
            _field("str", d["Name"]) + struct.pack(">q", d["Size"]) + d["ListH"] for d in v)
    if kind == "states":  # DatasetStateArray / DatasetStateEntry, core.go:187-206
        return struct.pack(">I", len(v)) + b"".join(struct.pack(">B", e["StateFlags"]) + _state(e["State"])
                                                     for e in v)
    if kind == "state":
        return _state(v)
    raise ValueError(kind)


def serialize(num: int, mtype: int, data: Optional[dict]) -> bytes:
    """ProtocolMessage.Serialize (protocol.go:184-203)."""
    out = header(num, mtype)
    schema = SCHEMA[mtype]
    if schema is not None:
        for name, kind in schema:
            out += _field(kind, data[name])
    return out


class _Reader:
    def __init__(self, buf: bytes):
        self.b, self.n = buf, 0

    def take(self, k: int) -> bytes:
        if self.n + k > len(self.b):
            raise EOFError
        v = self.b[self.n:self.n + k]
        self.n += k
        return v

    def fmt(self, f: str):
        return struct.unpack(f, self.take(struct.calcsize(f)))[0]


def _read(kind: str, r: _Reader):
    if kind == "u32":
        return r.fmt(">I")
    if kind == "b128":
        return r.take(16)
    if kind == "str":
        return r.take(r.fmt(">I"))
    if kind == "block":
        bid = r.take(16)
        links = [r.take(16) for _ in range(r.fmt(">I"))]
        dt = r.fmt(">B")
        return {"BlockID": bid, "Links": links, "DataType": dt, "Data": r.take(r.fmt(">I"))}
    if kind == "datasets":
        return [{"Name": _read("str", r), "Size": r.fmt(">q"), "ListH": r.take(16)} for _ in range(r.fmt(">I"))]
    if kind == "state":
        return {"StateID": r.take(16), "BlockID": r.take(16), "Size": r.fmt(">q"), "UniqueSize": r.fmt(">q")}
    if kind == "states":
        return [{"StateFlags": r.fmt(">B"), "State": _read("state", r)} for _ in range(r.fmt(">I"))]
    raise ValueError(kind)


def unserialize(buf: bytes) -> Tuple[int, int, Optional[dict], int]:
    """ProtocolMessage.Unserialize (protocol.go:204-264): (num, type, data,
    bytes used).  Unknown types raise, like the reference's panic."""
    r = _Reader(buf)
    num, mtype = r.fmt(">H"), r.fmt(">I")
    if mtype not in SCHEMA:
        raise ValueError(f"invalid protocol message received {mtype:x}")
    schema = SCHEMA[mtype]
    data = None if schema is None else {name: _read(kind, r) for name, kind in schema}
    return num, mtype, data, r.n


# the block-store exchange, byte for byte (used by the wire tools and tests)
def id_msg(num: int, mtype: int, block_id: bytes) -> bytes:
    """allo / read from the client, ACKN / READ from the server."""
    return serialize(num, mtype, {"BlockID": block_id})


def block_msg(num: int, mtype: int, block_id: bytes, links: Sequence[bytes], data_type: int, data: bytes) -> bytes:
    """writ / WRIT: MsgClientWriteBlock{Block} -> HashboxBlock.Serialize."""
    return serialize(num, mtype, {"Block": {"BlockID": block_id, "Links": list(links), "DataType": data_type,
                                            "Data": data}})


def error_msg(num: int, text: bytes) -> bytes:
    return serialize(num, ERROR & SM, {"ErrorMessage": text})


def greeting(num: int, version: int = 1) -> bytes:
    return serialize(num, GREETING, {"Version": version})


class LoopbackSink:
    """The server side of the block-store exchange, restated from
    server/server.go:160-202 (test infrastructure: it stands in for the Go
    server, which cannot be built here).  allo -> ACKN if the block is
    stored, else READ; writ -> VerifyBlock (UncompressData + HashData,
    pkg/core/block.go:152-174; every link must exist) -> store + ACKN, or
    ERRS "Unable to verify blockID"; quit -> QUIT and close.  Messages are
    read with this module's Unserialize restatement, not the product's
    parser."""

    def __init__(self, sock, preseed=()):
        import threading
        self.sock = sock
        self.store = set(bytes(x) for x in preseed)
        self.verified = 0
        self.failed = 0
        self.acked_allocs = 0
        self.reads = 0
        self.thread = threading.Thread(target=self._run, daemon=True)

    def start(self):
        self.thread.start()
        return self

    def _verify(self, block: dict) -> bool:
        import zlib
        from . import oracle as O
        try:
            data = zlib.decompress(block["Data"]) if block["DataType"] == ZLIB else block["Data"]
        except zlib.error:
            return False
        if any(bytes(link) not in self.store for link in block["Links"]):
            return False
        return O.py_block_id(data, block["Links"]) == block["BlockID"]

    def _run(self):
        buf = b""
        while True:
            chunk = self.sock.recv(1 << 20)
            if not chunk:
                return
            buf += chunk
            while True:
                try:
                    num, mtype, data, used = unserialize(buf)
                except EOFError:
                    break
                buf = buf[used:]
                if mtype == ALLOCATE:
                    bid = data["BlockID"]
                    if bid in self.store:
                        self.acked_allocs += 1
                        self.sock.sendall(id_msg(num, ACKNOWLEDGE & SM, bid))
                    else:
                        self.reads += 1
                        self.sock.sendall(id_msg(num, READ & SM, bid))
                elif mtype == WRITE:
                    b = data["Block"]
                    if self._verify(b):
                        self.verified += 1
                        self.store.add(b["BlockID"])
                        self.sock.sendall(id_msg(num, ACKNOWLEDGE & SM, b["BlockID"]))
                    else:
                        self.failed += 1
                        self.sock.sendall(error_msg(num, b"Unable to verify blockID"))
                elif mtype == GOODBYE:
                    self.sock.sendall(header(num, GOODBYE & SM))
                    return

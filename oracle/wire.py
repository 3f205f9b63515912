"""CPU restatement of the Hashbox wire messages used to store a block —
TEST INFRASTRUCTURE ONLY (tests/ and tools/ alone).

* ProtocolMessage.Serialize      pkg/core/protocol.go:184-203  (u16 Num, u32 Type, fields)
* message types / server mask    pkg/core/protocol.go:37-70
* MsgClientAllocateBlock etc.    pkg/core/protocol.go:100-131  (a 16-byte BlockID)
* HashboxBlock.Serialize         pkg/core/block.go:56-69       (id, links, type, len, data)
* big-endian integers            pkg/core/utils.go:73-88

Parity: pkg/core/protocol_test.go exercises these messages only as round trips
through the Go code itself (no byte fixtures), so the layouts are pinned by
source.
"""
from __future__ import annotations

import struct
from typing import Sequence

GREETING, GOODBYE = 0x68616C6F, 0x71756974
ALLOCATE, READ, WRITE, ACKNOWLEDGE, ERROR = 0x616C6C6F, 0x72656164, 0x77726974, 0x61636B6E, 0x65727273
SERVER_MASK = 0xDFDFDFDF
RAW, ZLIB = 0xFF, 0x01


def header(num: int, mtype: int) -> bytes:
    return struct.pack(">HI", num, mtype)


def id_msg(num: int, mtype: int, block_id: bytes) -> bytes:
    """allo / read from the client, ACKN / READ from the server."""
    return header(num, mtype) + block_id


def block_msg(num: int, mtype: int, block_id: bytes, links: Sequence[bytes], data_type: int, data: bytes) -> bytes:
    """writ / WRIT: MsgClientWriteBlock{Block} -> HashboxBlock.Serialize."""
    return (header(num, mtype) + block_id + struct.pack(">I", len(links)) + b"".join(links)
            + struct.pack(">BI", data_type, len(data)) + data)


def error_msg(num: int, text: bytes) -> bytes:
    return header(num, ERROR & SERVER_MASK) + struct.pack(">I", len(text)) + text


def greeting(num: int, version: int = 1) -> bytes:
    return header(num, GREETING) + struct.pack(">I", version)

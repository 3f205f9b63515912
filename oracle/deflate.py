"""zlib checker for the device block compressor — TEST INFRASTRUCTURE ONLY
(imported by ``tests/``, ``tools/`` validators and ``bench`` CPU legs alone).

The reference compresses a block with Go ``compress/zlib`` at
``DefaultCompression`` (pkg/core/block.go:176-184, level 6 = flate's default)
and the server only ever *inflates* it (block.go:113-131, 159-166).  So parity
for this path is not byte equality (the survey's §8f2 states the output need
not be bit-identical) but: every stream the device emits must be a complete,
valid RFC 1950 zlib stream whose inflation is exactly the block's data,
Adler-32 included.  The checker is CPython's ``zlib`` (the reference zlib
library, an independent RFC 1950/1951 implementation); the CPU baseline for
ratio and speed is the same library at level 6, standing in for Go's flate at
the same level (Go's toolchain is absent here).
"""
from __future__ import annotations

import zlib
from concurrent.futures import ThreadPoolExecutor
from typing import List, Sequence

LEVEL_DEFAULT = 6  # Go compress/flate DefaultCompression


def inflate_strict(stream: bytes) -> bytes:
    """Inflate one zlib stream; raises unless it is complete, checksummed and
    has no trailing bytes."""
    d = zlib.decompressobj(wbits=15)
    out = d.decompress(stream)
    out += d.flush()
    if not d.eof:
        raise ValueError("zlib stream not terminated (no final block / Adler-32)")
    if d.unused_data:
        raise ValueError(f"{len(d.unused_data)} bytes after the zlib stream")
    return out


def compress_ref(data: bytes, level: int = LEVEL_DEFAULT) -> bytes:
    return zlib.compress(data, level)


def compress_ref_mt(blocks: Sequence[bytes], threads: int, level: int = LEVEL_DEFAULT) -> List[bytes]:
    """zlib releases the GIL while compressing, so threads scale."""
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(lambda b: zlib.compress(b, level), blocks))


def inflate_mt(streams: Sequence[bytes], threads: int) -> List[bytes]:
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(zlib.decompress, streams))

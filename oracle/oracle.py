"""CPU oracle for the rollsum-split + block-ID path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg import this module.  The product package ``hashbox_amd`` never does: it
runs on the HIP library or fails.

Two restatements of the reference live here:

* ``liboracle`` — ctypes binding of ``oracle/hbx_oracle.c`` (plain C; the
  literal ``storeFile`` loop of hashback/store.go:111-185, RFC 1321 MD5,
  block framing pkg/core/block.go:96-111).
* ``py_store_file_literal`` — a pure-Python transliteration of the same loop
  (store.go:129-166) with the librsync rollsum (assumption A1),
  for small inputs only; it cross-checks the C oracle in tests.

Parity status: block IDs / MD5 are pinned by the HMAC-MD5 KATs
of pkg/core/core_test.go:23-30, by Python ``hashlib`` and by the "hello"
known answer; the split rule is pinned by source; the rollsum arithmetic
(third-party github.com/smtc/rollsum @ 39e98d252100, absent here) is
"reference-unpinned" — A1 is the librsync rolling checksum.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import struct
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

MIN_BLOCK_SIZE = 64 * 1024  # hashback/hashback.go:38
MAX_BLOCK_SIZE = 8 * 1024 * 1024  # hashback/hashback.go:37
CONTENT_TYPE_FILE_DATA = 2  # store.go:193
CONTENT_TYPE_FILE_CHAIN = 3  # store.go:189

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libhbxoracle.so")
_lib = None


def build() -> str:
    """Compile the C oracle (make -C oracle). Returns the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.hbxo_md5.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.hbxo_block_id.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint64, u8p]
        L.hbxo_chain_id.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.hbxo_window_digest.argtypes = [u8p, ctypes.c_uint64]
        L.hbxo_window_digest.restype = ctypes.c_uint32
        for fn in (L.hbxo_store_file, L.hbxo_store_file_fast):
            fn.argtypes = [u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_uint64, u8p,
                           ctypes.POINTER(ctypes.c_int32)]
            fn.restype = ctypes.c_int64
        L.hbxo_digest_all.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.hbxo_store_batch_mt.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p, u8p, u8p, u8p,
                                          ctypes.c_int]
        L.hbxo_hmac.argtypes = [u8p, ctypes.c_uint64, u8p, u8p]
        L.hbxo_deep_hmac.argtypes = [ctypes.c_int, u8p, ctypes.c_uint64, u8p, u8p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def max_chunks(n: int) -> int:
    """Every chunk but the last is >= MIN (store.go:130), so k <= n/MIN + 1."""
    return n // MIN_BLOCK_SIZE + 1


@dataclass
class FileResult:
    """What storeFile leaves behind (store.go:182-196): chunk ends, IDs, content."""
    cut_ends: np.ndarray  # uint64 [k]
    ids: np.ndarray  # uint8 [k, 16]
    content_type: int = 0
    content_id: bytes = b""

    @property
    def n_chunks(self) -> int:
        return int(self.cut_ends.shape[0])


def md5(data) -> bytes:
    a = _as_u8(data)
    out = np.zeros(16, np.uint8)
    lib().hbxo_md5(_ptr(a), a.size, _ptr(out))
    return out.tobytes()


def block_id(data, links: Sequence[bytes] = ()) -> bytes:
    a = _as_u8(data)
    ln = np.frombuffer(b"".join(links), np.uint8) if links else np.zeros(0, np.uint8)
    out = np.zeros(16, np.uint8)
    lib().hbxo_block_id(_ptr(ln), len(links), _ptr(a), a.size, _ptr(out))
    return out.tobytes()


def chain_id(ids: np.ndarray) -> bytes:
    ids = np.ascontiguousarray(ids, np.uint8).reshape(-1, 16)
    out = np.zeros(16, np.uint8)
    lib().hbxo_chain_id(_ptr(ids), ids.shape[0], _ptr(out))
    return out.tobytes()


def hmac(data: bytes, key: bytes, depth: int = 1) -> bytes:
    k = np.zeros(16, np.uint8)
    k[: len(key)] = np.frombuffer(key, np.uint8)[:16]
    a = _as_u8(data)
    out = np.zeros(16, np.uint8)
    lib().hbxo_deep_hmac(depth, _ptr(a), a.size, _ptr(k), _ptr(out))
    return out.tobytes()


def window_digest(window) -> int:
    a = _as_u8(window)
    return int(lib().hbxo_window_digest(_ptr(a), a.size))


def digest_all(data) -> np.ndarray:
    a = _as_u8(data)
    D = np.zeros(max(a.size, 1), np.uint32)
    lib().hbxo_digest_all(_ptr(a), a.size, _ptr(D))
    return D[: a.size]


def store_file(data, fast: bool = False) -> FileResult:
    """storeFile over an in-memory file (hashback/store.go:84-199)."""
    a = _as_u8(data)
    cap = max_chunks(a.size)
    cuts = np.zeros(cap, np.uint64)
    ids = np.zeros((cap, 16), np.uint8)
    cid = np.zeros(16, np.uint8)
    ct = ctypes.c_int32(0)
    fn = lib().hbxo_store_file_fast if fast else lib().hbxo_store_file
    k = fn(_ptr(a), a.size, _ptr(cuts), _ptr(ids), cap, _ptr(cid), ctypes.byref(ct))
    if k < 0:
        raise RuntimeError("oracle capacity overflow")
    return FileResult(cuts[:k].copy(), ids[:k].copy(), int(ct.value), cid.tobytes() if k else b"")


def store_batch_mt(files: List[np.ndarray], nthreads: int) -> List[FileResult]:
    """Files spread across ``nthreads`` OS threads, literal loop per file."""
    n = len(files)
    arrs = [_as_u8(f) for f in files]
    ptrs = np.array([_ptr(a) for a in arrs], np.uint64)
    lens = np.array([a.size for a in arrs], np.uint64)
    caps = np.array([max_chunks(a.size) for a in arrs], np.uint64)
    base = np.zeros(n, np.uint64)
    if n:
        base[1:] = np.cumsum(caps)[:-1]
    tot = int(caps.sum()) if n else 0
    cuts = np.zeros(max(tot, 1), np.uint64)
    ids = np.zeros((max(tot, 1), 16), np.uint8)
    counts = np.zeros(max(n, 1), np.int64)
    lib().hbxo_store_batch_mt(_ptr(ptrs), _ptr(lens), n, _ptr(cuts), _ptr(ids), _ptr(base),
                              _ptr(caps), _ptr(counts), int(nthreads))
    out = []
    for f in range(n):
        b, k = int(base[f]), int(counts[f])
        out.append(FileResult(cuts[b:b + k].copy(), ids[b:b + k].copy()))
    return out


# --------------------------------------------------------------------------
# Pure-Python transliteration (small inputs only) — independent of the C code.
# --------------------------------------------------------------------------
class _Rollsum:
    """librsync rollsum (assumption A1): Rollin/Rollout/Digest."""
    OFFSET = 31

    def __init__(self):
        self.count = self.s1 = self.s2 = 0

    def rollin(self, c):
        self.s1 += c + self.OFFSET
        self.s2 += self.s1
        self.count += 1

    def rollout(self, c):
        self.s1 -= c + self.OFFSET
        self.s2 -= self.count * (c + self.OFFSET)
        self.count -= 1

    def digest(self):
        return ((self.s2 << 16) | (self.s1 & 0xFFFF)) & 0xFFFFFFFF


def py_block_id(data: bytes, links: Sequence[bytes] = ()) -> bytes:
    """pkg/core/block.go:96-111 with hashlib (an MD5 independent of ours)."""
    h = hashlib.md5()
    h.update(struct.pack(">I", len(links)))
    for ln in links:
        h.update(ln)
    h.update(struct.pack(">I", len(data)))
    h.update(bytes(data))
    return h.digest()


def py_chain_id(ids: Sequence[bytes]) -> bytes:
    """hashback/hashback.go:162-170 serialisation hashed per store.go:188."""
    data = struct.pack(">II", 0x6663686E, len(ids)) + b"".join(i + bytes(16) for i in ids)
    return py_block_id(data, ids)


def py_store_file_literal(data: bytes):
    """store.go:111-185 transliterated; returns (cut_ends, ids, ctype, cid)."""
    data = bytes(data)
    n = len(data)
    off = 0
    cuts, ids = [], []
    while off < n:
        L = min(MAX_BLOCK_SIZE, n - off)
        buf = data[off:off + L]
        split = L
        if L > MIN_BLOCK_SIZE * 2:
            r = _Rollsum()
            maxd = 0
            rin = rout = 0
            while rin < L:
                if rin >= MIN_BLOCK_SIZE:
                    r.rollout(buf[rout])
                    rout += 1
                r.rollin(buf[rin])
                rin += 1
                if rin >= MIN_BLOCK_SIZE:
                    d = r.digest()
                    if d >= maxd:
                        maxd = d
                        split = rin
        cuts.append(off + split)
        ids.append(py_block_id(buf[:split]))
        off += split
    if len(ids) > 1:
        return cuts, ids, CONTENT_TYPE_FILE_CHAIN, py_chain_id(ids)
    if len(ids) == 1:
        return cuts, ids, CONTENT_TYPE_FILE_DATA, ids[0]
    return cuts, ids, 0, b""


# --------------------------------------------------------------------------
# Deterministic synthetic corpora (shared by tests / bench / fixtures).
# --------------------------------------------------------------------------
def random_bytes(n: int, seed: int) -> np.ndarray:
    """Uniform random bytes, numpy PCG64."""
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, n, dtype=np.uint8)


def zipf_corpus(n: int, seed: int, a: float = 1.1, pool: int = 64,
                seg_min: int = 64 * 1024, seg_max: int = 4 * 1024 * 1024) -> np.ndarray:
    """Duplicate-heavy bytes: segments drawn Zipf(a) from a pool of unique
    random segments (SURVEY.md §8d cfg 4)."""
    g = np.random.Generator(np.random.PCG64(seed))
    sizes = g.integers(seg_min, seg_max + 1, pool)
    segs = [g.integers(0, 256, int(s), dtype=np.uint8) for s in sizes]
    out = np.empty(n, np.uint8)
    pos = 0
    while pos < n:
        i = int(min(g.zipf(a), pool)) - 1
        s = segs[i]
        take = min(s.size, n - pos)
        out[pos:pos + take] = s[:take]
        pos += take
    return out

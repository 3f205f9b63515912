"""Host-side mirror of Hashback's chunking + block-ID interface on libhbxgpu.

Reference interface (fredli74/hashbox):
  * ``BackupSession.storeFile(path, entry)`` — hashback/store.go:84-199: splits
    a file by the rollsum rule and stores each chunk with
    ``Client.StoreData`` (pkg/core/client.go:556-560), whose
    ``NewHashboxBlock -> HashData`` (pkg/core/block.go:39-43, 96-111) yields
    the 16-byte BlockID; then sets ``entry.ContentType`` /
    ``entry.ContentBlockID`` (store.go:187-196).
  * ``HashboxBlock.HashData`` for blocks with links (chain/directory blocks).

:class:`Engine` exposes the same results — chunk end offsets, BlockIDs,
content type and content BlockID — computed on an MI355X.  Every call goes
through the C-ABI (include/hbxgpu.h); there is no CPU fallback, and errors
raise :class:`HbxError` (the reference panics via core.Abort,
pkg/core/utils.go:22-37).
"""
from __future__ import annotations

import ctypes
import gc
import os
import sys
import time
from collections import deque
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Union

import numpy as np

from . import _lib

MIN_BLOCK_SIZE = 64 * 1024  # hashback/hashback.go:38
MAX_BLOCK_SIZE = 8 * 1024 * 1024  # hashback/hashback.go:37
CONTENT_TYPE_FILE_DATA = 2  # store.go:193
CONTENT_TYPE_FILE_CHAIN = 3  # store.go:189
ARENA_ALIGN = 16
ARENA_SLACK = 64

BytesLike = Union[bytes, bytearray, memoryview, np.ndarray]


class HbxError(RuntimeError):
    """A non-zero status from libhbxgpu."""


def max_chunks(n: int) -> int:
    return n // MIN_BLOCK_SIZE + 1


@dataclass(slots=True)
class FileChunks:
    """What storeFile records for one file."""
    cut_ends: np.ndarray  # uint64 [k]: chunk i = [cut_ends[i-1], cut_ends[i])
    ids: np.ndarray  # uint8 [k, 16]: BlockID per chunk (core.Byte128)
    content_type: int  # 2 FileData, 3 FileChain (0 for an empty file)
    content_id: bytes  # entry.ContentBlockID
    zstreams: Optional[list] = None  # zlib stream per chunk, uint8 views (store_paths(compress=True))
    errno: int = 0  # store_paths(skip_unreadable=True): the errno of a file skipped (no chunks), else 0

    @property
    def n_chunks(self) -> int:
        return int(self.cut_ends.shape[0])

    def chunk_bounds(self):
        starts = np.concatenate([[0], self.cut_ends[:-1]]).astype(np.uint64)
        return starts, self.cut_ends


def _u8(data: BytesLike) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data.reshape(-1).view(np.uint8))
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def _p(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _huge_host_buffer(nbytes: int) -> np.ndarray:
    """A host byte buffer the library fills once (the compressed streams of a
    whole store_paths call): an anonymous mapping advised for transparent
    huge pages, so its first touch costs one fault per 2 MiB instead of per
    4 KiB (60 GB of 4 KiB first-touch faults cost ~1.4 s on 16 threads)."""
    import mmap
    m = mmap.mmap(-1, max(nbytes, 1), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        try:
            m.madvise(mmap.MADV_HUGEPAGE)
        except OSError:
            pass
    return np.frombuffer(m, np.uint8)  # the array keeps the mapping alive


class Engine:
    """One MI355X (one HIP stream) running the chunk + block-ID path."""

    def __init__(self, device: int = 0, tile_iters: Optional[int] = None,
                 md5_slice: Optional[int] = None, join_lag: Optional[int] = None,
                 k3_period: Optional[int] = None):
        self._L = _lib.load()
        self._ctx = ctypes.c_void_p()
        rc = self._L.hbx_ctx_create(int(device), ctypes.byref(self._ctx))
        if rc != 0:
            raise HbxError(f"hbx_ctx_create(device={device}) failed: {_lib.ERRORS.get(rc, rc)}")
        self.device = device
        self._pending = deque()
        self.wait_s = 0.0
        self.last_call_s = 0.0
        if tile_iters is not None:
            self._check(self._L.hbx_set_tile_iters(self._ctx, int(tile_iters)), "set_tile_iters")
        if md5_slice is not None:
            self.set_md5_slice(md5_slice)
        if join_lag is not None:
            self.set_join_lag(join_lag)
        if k3_period is not None:
            self.set_k3_period(k3_period)

    # ----------------------------------------------------------- plumbing --
    def _after_producer(self):
        """The engine's HIP streams do not wait for other streams: device data
        written on torch's current stream (e.g. a tensor just filled) must be
        complete before the engine reads it.  The device-pointer entry points
        call this first; the dependency is a GPU-side event wait
        (hbx_after_stream), so the host never blocks and can submit batches
        ahead of the device."""
        t = sys.modules.get("torch")
        if t is not None and t.cuda.is_initialized():
            s = t.cuda.current_stream(self.device)
            self._check(self._L.hbx_after_stream(self._ctx, ctypes.c_void_p(int(s.cuda_stream))),
                        "hbx_after_stream")

    def close(self):
        if self._ctx:
            self._L.hbx_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str):
        if rc != 0:
            msg = self._L.hbx_last_error(self._ctx)
            raise HbxError(f"{what}: {_lib.ERRORS.get(rc, rc)}: "
                           f"{msg.decode() if msg else ''}")

    @staticmethod
    def _alloc_out(lens: Sequence[int]):
        caps = (np.asarray(lens, np.uint64).reshape(-1) // np.uint64(MIN_BLOCK_SIZE) + np.uint64(1)
                if len(lens) else np.zeros(0, np.uint64))
        base = np.zeros(len(lens), np.uint64)
        if len(lens):
            base[1:] = np.cumsum(caps)[:-1]
        tot = int(caps.sum()) if len(lens) else 0
        cuts = np.zeros(max(tot, 1), np.uint64)
        ids = np.zeros((max(tot, 1), 16), np.uint8)
        sums = (_lib.FileSummary * max(len(lens), 1))()
        return caps, base, cuts, ids, sums

    @staticmethod
    def _unpack(lens, caps, base, cuts, ids, sums) -> List[FileChunks]:
        # one structured view of the summaries; each file's cut ends and ids
        # are views into the per-call output arrays (no per-file copies:
        # 100 k files unpack in ~0.15 s instead of ~0.4 s)
        n = len(lens)
        if n == 0:
            return []
        sv = np.ctypeslib.as_array(sums)[:n]
        k = sv["n_chunks"].astype(np.int64)
        starts = base[:n].astype(np.int64).tolist()
        ks = k.tolist()
        types = sv["content_type"].tolist()
        cid = np.ascontiguousarray(sv["content_id"]).tobytes()
        # the cyclic collector would run dozens of passes over 100 k new objects
        was = gc.isenabled()
        gc.disable()
        try:
            return [FileChunks(cuts[b:b + kk], ids[b:b + kk], t, cid[16 * f:16 * f + 16] if kk else b"")
                    for f, (b, kk, t) in enumerate(zip(starts, ks, types))]
        finally:
            if was:
                gc.enable()

    # -------------------------------------------------------------- API ----
    def chunk_hash(self, data: BytesLike) -> FileChunks:
        """storeFile over one in-memory file (store.go:111-196)."""
        return self.chunk_hash_batch([data])[0]

    def chunk_hash_batch(self, files: Sequence[BytesLike]) -> List[FileChunks]:
        arrs = [_u8(f) for f in files]
        lens = np.array([a.size for a in arrs], np.uint64)
        ptrs = np.array([_p(a) for a in arrs], np.uint64)
        caps, base, cuts, ids, sums = self._alloc_out(lens)
        self._check(self._L.hbx_chunk_hash_batch(self._ctx, len(arrs), _p(ptrs), _p(lens),
                                                 _p(cuts), _p(ids), _p(base), _p(caps), sums),
                    "hbx_chunk_hash_batch")
        return self._unpack(lens, caps, base, cuts, ids, sums)

    def chunk_hash_device(self, d_arena: int, offs: Sequence[int], lens: Sequence[int]
                          ) -> List[FileChunks]:
        """Files resident in device memory (pointer ``d_arena``, e.g. a torch
        uint8 tensor's ``data_ptr()``).  Offsets 16-B aligned; each file must be
        followed by >= 64 readable bytes."""
        self._after_producer()
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        caps, base, cuts, ids, sums = self._alloc_out(lens)
        self._check(self._L.hbx_chunk_hash_device(self._ctx, ctypes.c_void_p(int(d_arena)), len(lens),
                                                  _p(offs), _p(lens), _p(cuts), _p(ids), _p(base),
                                                  _p(caps), sums), "hbx_chunk_hash_device")
        return self._unpack(lens, caps, base, cuts, ids, sums)

    def submit_device(self, d_arena: int, offs: Sequence[int], lens: Sequence[int]):
        """Enqueue a device-resident batch and return at once.  Any number of
        batches may be in flight; :meth:`wait` completes the oldest.  The
        arena must stay untouched until then."""
        self._after_producer()
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        t0 = time.perf_counter()
        caps, base, cuts, ids, sums = self._alloc_out(lens)
        t1 = time.perf_counter()
        self.alloc_s = t1 - t0  # (bench diagnostics: host output arrays of this submit)
        self._check(self._L.hbx_submit_device(self._ctx, ctypes.c_void_p(int(d_arena)), len(lens),
                                              _p(offs), _p(lens), _p(cuts), _p(ids), _p(base),
                                              _p(caps), sums), "hbx_submit_device")
        self._pending.append((offs, lens, caps, base, cuts, ids, sums))

    def wait(self):
        """Results of the oldest submitted batch ([] if none is pending): a
        list of FileChunks for a chunking batch, (ids, ok, n_bad) for a
        verify batch."""
        if not self._pending:
            return []
        item = self._pending.popleft()
        t = time.perf_counter()
        rc = self._L.hbx_wait(self._ctx)
        self.wait_s += time.perf_counter() - t  # time inside hbx_wait (bench diagnostics)
        self._check(rc, "hbx_wait")
        if isinstance(item[0], str):  # ("verify", ...)
            _, n, ids, ok, bad, keep = item
            return ids[:n], (ok[:n].astype(bool) if keep[1] is not None else None), int(bad.value)
        offs, lens, caps, base, cuts, ids, sums = item
        return self._unpack(lens, caps, base, cuts, ids, sums)

    def verify_submit_device(self, d_arena: int, offs: Sequence[int], lens: Sequence[int],
                             links: Optional[Sequence[Sequence[bytes]]] = None,
                             expect: Optional[Sequence[bytes]] = None):
        """Pipelined VerifyBlock of device-resident blocks (hbx_verify_submit_device):
        returns at once; :meth:`wait` (FIFO with chunking batches) returns
        (ids, ok, n_bad)."""
        self._after_producer()
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        n = int(lens.size)
        links_a, base, counts = self._links_arrays(links, n)
        ids = np.zeros((max(n, 1), 16), np.uint8)
        exp = None
        if expect is not None:
            exp = np.ascontiguousarray(np.frombuffer(b"".join(bytes(e) for e in expect), np.uint8))
            if exp.size != 16 * n:
                raise ValueError("expect must hold one 16-byte ID per block")
        ok = np.zeros(max(n, 1), np.uint8)
        bad = ctypes.c_uint64(0)
        self._check(self._L.hbx_verify_submit_device(
            self._ctx, ctypes.c_void_p(int(d_arena)), n, _p(offs), _p(lens),
            _p(links_a) if links_a is not None else None, _p(base) if base is not None else None,
            _p(counts) if counts is not None else None, _p(ids), _p(exp) if exp is not None else None,
            _p(ok), ctypes.byref(bad)), "hbx_verify_submit_device")
        # everything the library writes or reads until the wait stays alive here
        self._pending.append(("verify", n, ids, ok, bad, (offs, exp, lens)))

    def pending(self) -> int:
        n = self._L.hbx_pending(self._ctx)
        if n < 0:
            self._check(n, "hbx_pending")
        return int(n)

    def set_md5_slice(self, blocks: int):
        """MD5 blocks per chain per K3 launch (0 = unlimited)."""
        self._check(self._L.hbx_set_md5_slice(self._ctx, int(blocks)), "hbx_set_md5_slice")

    def input_after_oldest(self):
        """The next input copy / batch may reuse the oldest pending batch's
        device memory: a GPU-side wait for its hashing to finish
        (hbx_input_after_oldest)."""
        self._check(self._L.hbx_input_after_oldest(self._ctx), "hbx_input_after_oldest")

    def input_fence(self, stream: Optional[int] = None):
        """Enqueue the pending wait of :meth:`input_after_oldest` now, and on
        ``stream`` (a raw hipStream_t handle) too: needed before the caller
        writes the old batch's memory with its own work (hbx_input_fence)."""
        self._check(self._L.hbx_input_fence(self._ctx, ctypes.c_void_p(int(stream) if stream else 0)),
                    "hbx_input_fence")

    def set_k3_probe(self, on: bool = True):
        """Diagnostics: per-wave records of every K3 launch (hbx_set_k3_probe)."""
        self._check(self._L.hbx_set_k3_probe(self._ctx, int(bool(on))), "hbx_set_k3_probe")

    def set_join_lag(self, lag: int):
        """Submits between a batch's own and the MD5 launch its chains join
        (1..4; 2 gives a small batch's scan a whole extra step)."""
        self._check(self._L.hbx_set_join_lag(self._ctx, int(lag)), "hbx_set_join_lag")

    def set_k3_period(self, period: int):
        """One K3 launch every ``period`` submits (1..8) with ``period`` x the
        slice per chain: small batches pay the launch's start-up and tail once
        per period (hbx_set_k3_period)."""
        self._check(self._L.hbx_set_k3_period(self._ctx, int(period)), "hbx_set_k3_period")

    def k3_wave_times(self) -> np.ndarray:
        """Diagnostics (:meth:`set_k3_probe`): per-wave records of the
        latest K3 launch, shape (waves, 8): start, start-up end | XCC << 56,
        end (100 MHz ticks), R | max count << 16 | HW_ID << 32, then the
        first group's cooperative phase: s_memtime at its start and end,
        s_memrealtime at its end, blocks per chain (R - 1)."""
        n = ctypes.c_uint32(0)
        self._check(self._L.hbx_k3_wave_times(self._ctx, None, 0, ctypes.byref(n)), "hbx_k3_wave_times")
        out = np.zeros((max(n.value, 1), 8), np.uint64)
        self._check(self._L.hbx_k3_wave_times(self._ctx, _p(out), n.value, ctypes.byref(n)), "hbx_k3_wave_times")
        return out[:n.value]

    def knobs(self) -> dict:
        """The context's effective pipeline knobs (hbx_knobs), including
        whether HBX_* A/B switches were honoured (only with HBX_AB=1)."""
        import json
        buf = ctypes.create_string_buffer(4096)
        self._check(self._L.hbx_knobs(self._ctx, buf, len(buf)), "hbx_knobs")
        return json.loads(buf.value.decode())

    def reserve(self, batches: int, files: int, nbytes: int):
        """Pre-size the pipeline for ``batches`` batches in flight of up to
        ``files`` files / ``nbytes`` bytes each, so the steady state never
        allocates (an allocation drains both streams)."""
        self._check(self._L.hbx_reserve(self._ctx, int(batches), int(files), int(nbytes)),
                    "hbx_reserve")

    def plan_pipeline(self, **kw) -> dict:
        """hbx_plan_pipeline on this context (free_bytes=0: the device's free
        memory now); see the module function :func:`plan_pipeline`."""
        return plan_pipeline(engine=self, **kw)

    def apply_plan(self, plan: dict, files: int, nbytes: int):
        """hbx_apply_plan: the plan's slice, join lag and K3 period, and R + 2
        reserved batches of up to `files` files and `nbytes` bytes."""
        pp = _lib.PipelinePlan(**{k: int(plan[k]) for k in _PLAN_KEYS})
        self._check(self._L.hbx_apply_plan(self._ctx, ctypes.byref(pp), int(files), int(nbytes)), "hbx_apply_plan")

    def stage_totals(self, reset: bool = False):
        """Cumulative device ms and launch counts per kernel: K1, K2, plan, K3, K4."""
        ms = (ctypes.c_double * 5)()
        n = (ctypes.c_uint64 * 5)()
        self._check(self._L.hbx_stage_totals(self._ctx, ms, n, int(bool(reset))), "hbx_stage_totals")
        return np.array(list(ms), np.float64), np.array(list(n), np.int64)

    def block_id(self, data: BytesLike, links: Sequence[bytes] = ()) -> bytes:
        """HashboxBlock.HashData (pkg/core/block.go:96-111) on the device."""
        a = _u8(data)
        ln = np.frombuffer(b"".join(bytes(x) for x in links), np.uint8) if links else \
            np.zeros(0, np.uint8)
        out = np.zeros(16, np.uint8)
        self._check(self._L.hbx_block_id(self._ctx, _p(ln), len(links), _p(a), a.size, _p(out)),
                    "hbx_block_id")
        return out.tobytes()

    def md5(self, data: BytesLike) -> bytes:
        """core.Hash (pkg/core/core.go:46-48): MD5 of the raw bytes on the device."""
        a = _u8(data)
        out = np.zeros(16, np.uint8)
        self._check(self._L.hbx_md5(self._ctx, _p(a), a.size, _p(out)), "hbx_md5")
        return out.tobytes()

    def hmac(self, data: bytes, key: bytes) -> bytes:
        """core.Hmac (pkg/core/core.go:51-68) with the device MD5 as the hash."""
        k = (bytes(key) + bytes(16))[:16] + bytes(48)  # Byte128 key, zero-padded to md5.BlockSize
        inner = self.md5(bytes(b ^ 0x36 for b in k) + bytes(data))
        return self.md5(bytes(b ^ 0x5C for b in k) + inner)

    def deep_hmac(self, depth: int, data: bytes, key: bytes) -> bytes:
        """core.DeepHmac (pkg/core/core.go:70-80): depth rounds of Hmac."""
        h, d = bytes(16), bytes(data)
        for _ in range(depth):
            h = d = self.hmac(d, key)
        return h

    @staticmethod
    def _links_arrays(links_per_block: Optional[Sequence[Sequence[bytes]]], n: int):
        if not links_per_block or not any(len(x) for x in links_per_block):
            return None, None, None
        counts = np.array([len(x) for x in links_per_block], np.uint32)
        base = np.zeros(n, np.uint64)
        base[1:] = np.cumsum(counts.astype(np.uint64))[:-1]
        flat = np.frombuffer(b"".join(bytes(l) for x in links_per_block for l in x), np.uint8)
        if flat.size != 16 * int(counts.sum()):
            raise ValueError("every link must be a 16-byte block ID")
        return np.ascontiguousarray(flat), base, counts

    def _verify(self, fn, lead_args, n, links, expect):
        links_a, base, counts = self._links_arrays(links, n)
        ids = np.zeros((max(n, 1), 16), np.uint8)
        exp = None
        if expect is not None:
            exp = np.ascontiguousarray(np.frombuffer(b"".join(bytes(e) for e in expect), np.uint8))
            if exp.size != 16 * n:
                raise ValueError("expect must hold one 16-byte ID per block")
        ok = np.zeros(max(n, 1), np.uint8)
        bad = ctypes.c_uint64(0)
        self._check(fn(self._ctx, *lead_args,
                       _p(links_a) if links_a is not None else None,
                       _p(base) if base is not None else None,
                       _p(counts) if counts is not None else None,
                       _p(ids), _p(exp) if exp is not None else None, _p(ok), ctypes.byref(bad)),
                    fn.__name__)
        return ids[:n], (ok[:n].astype(bool) if expect is not None else None), int(bad.value)

    def verify_blocks(self, blocks: Sequence[BytesLike], links: Optional[Sequence[Sequence[bytes]]] = None,
                      expect: Optional[Sequence[bytes]] = None):
        """HashboxBlock.HashData / VerifyBlock (pkg/core/block.go:96-111,
        152-174) for many uncompressed blocks at once.  Returns (ids [n,16],
        ok [n] bool or None, number of mismatches)."""
        arrs = [_u8(b) for b in blocks]
        n = len(arrs)
        lens = np.array([a.size for a in arrs], np.uint64)
        ptrs = np.array([_p(a) for a in arrs], np.uint64)
        return self._verify(self._L.hbx_verify_blocks, (n, _p(ptrs), _p(lens)), n, links, expect)

    def verify_blocks_device(self, d_arena: int, offs: Sequence[int], lens: Sequence[int],
                             links: Optional[Sequence[Sequence[bytes]]] = None,
                             expect: Optional[Sequence[bytes]] = None):
        """The same for blocks resident in device memory (each followed by
        >= 64 readable bytes)."""
        self._after_producer()
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        n = int(lens.size)
        return self._verify(self._L.hbx_verify_blocks_device,
                            (ctypes.c_void_p(int(d_arena)), n, _p(offs), _p(lens)), n, links, expect)

    def deflate_bound(self, n: int) -> int:
        """Largest zlib stream hbx_deflate_blocks* produces for n bytes."""
        return int(self._L.hbx_deflate_bound(int(n)))

    def deflate_blocks(self, blocks: Sequence[BytesLike]) -> List[bytes]:
        """HashboxBlock.CompressData (pkg/core/block.go:133-150, 176-184) for
        many blocks at once: one zlib stream per block, coded on the device."""
        arrs = [_u8(b) for b in blocks]
        n = len(arrs)
        if n == 0:
            return []
        lens = np.array([a.size for a in arrs], np.uint64)
        caps = np.array([self.deflate_bound(int(x)) for x in lens], np.uint64)
        outs = [np.empty(int(c), np.uint8) for c in caps]
        dptr = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
        optr = (ctypes.c_void_p * n)(*[o.ctypes.data for o in outs])
        olen = np.zeros(n, np.uint64)
        self._check(self._L.hbx_deflate_blocks(self._ctx, n, dptr, _p(lens), optr, _p(caps), _p(olen)),
                    "hbx_deflate_blocks")
        return [o[:int(k)].tobytes() for o, k in zip(outs, olen)]

    def deflate_blocks_device(self, d_arena: int, offs: Sequence[int], lens: Sequence[int], d_out: int,
                              out_offs: Sequence[int], out_caps: Sequence[int]) -> np.ndarray:
        """Device form: block i = d_arena[offs[i] ..+lens[i]) -> zlib stream at
        d_out[out_offs[i] ..]; returns the stream lengths."""
        self._after_producer()
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        oo = np.ascontiguousarray(out_offs, np.uint64)
        oc = np.ascontiguousarray(out_caps, np.uint64)
        olen = np.zeros(max(lens.size, 1), np.uint64)
        self._check(self._L.hbx_deflate_blocks_device(self._ctx, ctypes.c_void_p(int(d_arena)), lens.size,
                                                      _p(offs), _p(lens), ctypes.c_void_p(int(d_out)), _p(oo),
                                                      _p(oc), _p(olen)), "hbx_deflate_blocks_device")
        return olen[:lens.size]

    def inflate_blocks_device(self, d_in: int, in_offs: Sequence[int], in_lens: Sequence[int], d_out: int,
                              out_offs: Sequence[int], out_caps: Sequence[int]):
        """HashboxBlock.UncompressData (block.go:113-131) of many zlib streams on
        the device: returns (out_lens, status) (status 0 = ok)."""
        self._after_producer()
        io = np.ascontiguousarray(in_offs, np.uint64)
        il = np.ascontiguousarray(in_lens, np.uint64)
        oo = np.ascontiguousarray(out_offs, np.uint64)
        oc = np.ascontiguousarray(out_caps, np.uint64)
        n = int(il.size)
        ol = np.zeros(max(n, 1), np.uint64)
        st = np.zeros(max(n, 1), np.uint32)
        self._check(self._L.hbx_inflate_blocks_device(self._ctx, ctypes.c_void_p(int(d_in)), n, _p(io), _p(il),
                                                      ctypes.c_void_p(int(d_out)), _p(oo), _p(oc), _p(ol),
                                                      _p(st)), "hbx_inflate_blocks_device")
        return ol[:n], st[:n]

    def inflate_blocks(self, streams: Sequence[BytesLike], caps: Sequence[int]):
        """Host convenience: inflate zlib streams on the device; returns
        (list of bytes or None per stream, status array)."""
        import torch
        arrs = [_u8(z) for z in streams]
        n = len(arrs)
        if n == 0:
            return [], np.zeros(0, np.uint32)
        io = np.zeros(n, np.uint64)
        pos = 0
        for i, a in enumerate(arrs):
            io[i] = pos
            pos += (a.size + 255) // 256 * 256
        host = np.zeros(pos + 64, np.uint8)
        for i, a in enumerate(arrs):
            host[int(io[i]):int(io[i]) + a.size] = a
        oc = np.ascontiguousarray(caps, np.uint64)
        oo = np.zeros(n, np.uint64)
        oo[1:] = np.cumsum((oc[:-1] + 255) // 256 * 256)
        dev = torch.device("cuda", self.device)  # this engine's GPU, not torch's current one
        d_in = torch.from_numpy(host).to(dev)
        d_out = torch.zeros(int(oo[-1] + oc[-1]) + 64, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        ol, st = self.inflate_blocks_device(d_in.data_ptr(), io, [a.size for a in arrs], d_out.data_ptr(), oo, oc)
        out = d_out.cpu().numpy()
        return [out[int(oo[i]):int(oo[i] + ol[i])].tobytes() if st[i] == 0 else None for i in range(n)], st

    def memcpy_h2d_async(self, d_dst: int, h_src: int, nbytes: int):
        """Enqueue an H2D copy on this engine's stream (pinned source)."""
        self._check(self._L.hbx_memcpy_h2d_async(self._ctx, ctypes.c_void_p(int(d_dst)),
                                                 ctypes.c_void_p(int(h_src)), int(nbytes)),
                    "hbx_memcpy_h2d_async")

    def store_paths(self, paths: Sequence[Union[str, os.PathLike]], io_threads: int = 16,
                    batch_bytes: int = 1 << 30, compress: bool = False,
                    on_batch: Optional[Callable[[int, int], None]] = None,
                    on_files: Optional[Callable[[int, List[FileChunks]], None]] = None,
                    sizes: Optional[Sequence[int]] = None,
                    skip_unreadable: bool = False) -> List[FileChunks]:
        """storeFile for many files on disk, end to end: the library reads them
        into pinned memory on ``io_threads`` threads and overlaps reading the
        next batch with the copy + kernels of the current one.  With
        ``compress`` every chunk is also zlib-compressed on the device
        (HashboxBlock.CompressData, the client's send path) and returned in
        ``FileChunks.zstreams``.  ``on_batch(first, count)`` (compress only)
        runs on this thread as soon as files [first, first+count) have their
        ids, summaries and zlib streams written (hbx_store_paths_zcb), so a
        sender can ship them while later batches are still read and hashed.
        ``on_files(first, files)`` is the same callback handed the finished
        FileChunks (ids, cut ends, zlib stream views) of those files.
        ``sizes`` are the files' byte sizes when the caller already has them
        (storeFile takes the walker's FileEntry with FileSize, store.go:84,
        247); otherwise each path is stat'ed here.  A file shorter than its
        size fails the call (HBX_ERR_IO); bytes past it are not read.  With
        ``skip_unreadable`` (hbx_store_paths_status) a file the reference skips
        without stopping the walk -- open() failing (store.go:101-103,
        221-224) or a read failing with EBADF (minorPathError,
        hashback_unix.go:57-63) -- comes back with no chunks and its errno in
        ``FileChunks.errno``, and the rest of its batch is stored; any other
        read error still fails the call.  ``last_call_s`` holds the library
        call's wall seconds."""
        if (on_batch is not None or on_files is not None) and not compress:
            raise ValueError("on_batch / on_files need compress=True (hbx_store_paths_zcb)")
        enc = [os.fsencode(p) for p in paths]
        if sizes is None:
            lens = np.array([os.stat(p).st_size for p in enc], np.uint64)
        else:
            lens = np.array(sizes, np.uint64).reshape(-1)
            if lens.size != len(enc):
                raise ValueError("sizes must have one entry per path")
        arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        caps, base, cuts, ids, sums = self._alloc_out(lens)
        status = np.zeros(max(len(enc), 1), np.int32) if skip_unreadable else None

        def with_status(res):
            if status is not None:
                for r, e in zip(res, status[:len(res)].tolist()):
                    r.errno = int(e)
            return res

        if not compress:
            t0 = time.perf_counter()
            if status is None:
                self._check(self._L.hbx_store_paths(self._ctx, len(enc), ctypes.cast(arr, ctypes.c_void_p),
                                                    _p(lens), _p(cuts), _p(ids), _p(base), _p(caps), sums,
                                                    int(io_threads), int(batch_bytes)), "hbx_store_paths")
            else:
                self._check(self._L.hbx_store_paths_status(
                    self._ctx, len(enc), ctypes.cast(arr, ctypes.c_void_p), _p(lens), _p(cuts), _p(ids), _p(base),
                    _p(caps), sums, _p(status), int(io_threads), int(batch_bytes), None, None, None, None, None,
                    None), "hbx_store_paths_status")
            self.last_call_s = time.perf_counter() - t0
            return with_status(self._unpack(lens, caps, base, cuts, ids, sums))
        fb = np.array([self._L.hbx_deflate_file_bound(int(x)) for x in lens], np.uint64)
        zbase = np.zeros(max(lens.size, 1), np.uint64)
        if lens.size > 1:
            zbase[1:lens.size] = np.cumsum(fb[:-1])
        zout = _huge_host_buffer(int(fb.sum()) + 16)
        zoff = np.zeros(max(int(caps.sum()), 1), np.uint64)
        zlen = np.zeros_like(zoff)
        zargs = (self._ctx, len(enc), ctypes.cast(arr, ctypes.c_void_p), _p(lens), _p(cuts), _p(ids),
                 _p(base), _p(caps), sums, int(io_threads), int(batch_bytes), _p(zout), _p(zbase),
                 _p(zoff), _p(zlen))
        def view(f: int) -> FileChunks:  # file f's results, as soon as its batch is reported
            s = sums[f]
            k, b = int(s.n_chunks), int(base[f])
            r = FileChunks(cuts[b:b + k].copy(), ids[b:b + k].copy(), int(s.content_type),
                           bytes(s.content_id) if k else b"")
            r.zstreams = [zout[int(zoff[b + i]):int(zoff[b + i] + zlen[b + i])] for i in range(k)]
            if status is not None:  # written when the file was read, before its batch was reported
                r.errno = int(status[f])
            return r

        t0 = time.perf_counter()
        if status is not None:  # the same with per-file outcomes (hbx_store_paths_status)
            zargs_st = zargs[:9] + (_p(status),) + zargs[9:]
        if on_batch is None and on_files is None:
            if status is None:
                self._check(self._L.hbx_store_paths_z(*zargs), "hbx_store_paths_z")
            else:
                self._check(self._L.hbx_store_paths_status(*zargs_st, None, None), "hbx_store_paths_status")
        else:
            raised = []

            def ready(_user, first, count):
                if raised:
                    return
                try:
                    if on_batch is not None:
                        on_batch(int(first), int(count))
                    if on_files is not None:
                        on_files(int(first), [view(f) for f in range(int(first), int(first + count))])
                except BaseException as e:  # never unwind through C
                    raised.append(e)
            cb = _lib.BATCH_READY(ready)
            if status is None:
                self._check(self._L.hbx_store_paths_zcb(*zargs, ctypes.cast(cb, ctypes.c_void_p), None),
                            "hbx_store_paths_zcb")
            else:
                self._check(self._L.hbx_store_paths_status(*zargs_st, ctypes.cast(cb, ctypes.c_void_p), None),
                            "hbx_store_paths_status")
            if raised:
                raise raised[0]
        self.last_call_s = time.perf_counter() - t0
        res = with_status(self._unpack(lens, caps, base, cuts, ids, sums))
        for f, r in enumerate(res):
            b = int(base[f])
            r.zstreams = [zout[int(zoff[b + i]):int(zoff[b + i] + zlen[b + i])]  # views, no copy
                          for i in range(r.n_chunks)]
        return res

    def host_call_max(self, reset: bool = False) -> np.ndarray:
        """hbx_host_call_max: ms of the slowest single H2D copy call and the
        slowest single submit since the last reset."""
        a = (ctypes.c_double * 2)()
        self._check(self._L.hbx_host_call_max(self._ctx, a, int(reset)), "hbx_host_call_max")
        return np.array(list(a))

    def io_times(self, reset: bool = False) -> np.ndarray:
        """store_paths host seconds: reading files, waiting for batches to be
        collected (arena reuse and the final drain), waiting for a pinned
        slot's copy (cumulative)."""
        s = (ctypes.c_double * 3)()
        self._check(self._L.hbx_io_times(self._ctx, s, int(bool(reset))), "hbx_io_times")
        return np.array(list(s), np.float64)

    def store_file(self, path: Union[str, os.PathLike]) -> FileChunks:
        """storeFile(path) for a regular file on disk (store.go:84-199)."""
        with open(path, "rb") as fh:
            data = np.fromfile(fh, dtype=np.uint8)
        return self.chunk_hash(data)

    def stage_times(self) -> np.ndarray:
        """Device ms of the last collected batch: K1, K2, plan + first K3
        launch, later K3 launches + K4, total (synchronous calls: K3 in [2],
        K4 in [3])."""
        ms = (ctypes.c_float * 5)()
        self._check(self._L.hbx_stage_times(self._ctx, ms), "hbx_stage_times")
        return np.array(list(ms), np.float64)


_PLAN_KEYS = ("resident", "md5_slice", "join_lag", "lead", "k3_period", "launches_per_batch", "hbm_bytes")


def plan_pipeline(n_files: int, arena_bytes: int, longest_file: int, free_bytes: int = 0, hbm_frac: float = 0.95,
                  ranks_per_device: int = 1, steps: int = 0, arenas: int = 0, md5_slice: int = -1,
                  join_lag: int = 0, lead: int = -1, k3_period: int = 0, host_input: bool = False,
                  engine: Optional["Engine"] = None) -> dict:
    """The pipeline's operating point from the library (hbx_plan_pipeline,
    include/hbxgpu.h): resident batches R, MD5 slice, join lag, lead, K3
    period, launches per batch and the HBM the arenas take.  Pure host
    arithmetic when free_bytes > 0 (no GPU needed); with free_bytes=0 an
    engine must be given (its device's free memory).  Raises ValueError for
    an impossible request."""
    L = _lib.load()
    q = _lib.PlanRequest(n_files=int(n_files), arena_bytes=int(arena_bytes), longest_file=int(longest_file),
                         free_bytes=int(free_bytes), hbm_frac=float(hbm_frac),
                         ranks_per_device=int(ranks_per_device), steps=int(steps), arenas=int(arenas),
                         md5_slice=int(md5_slice), join_lag=int(join_lag), lead=int(lead),
                         k3_period=int(k3_period), flags=_lib.PLAN_HOST_INPUT if host_input else 0)
    p = _lib.PipelinePlan()
    ctx = engine._ctx if engine is not None else None
    rc = L.hbx_plan_pipeline(ctx, ctypes.byref(q), ctypes.byref(p))
    if rc != 0:
        msg = L.hbx_last_error(ctx).decode()
        raise ValueError(f"hbx_plan_pipeline: {_lib.ERRORS.get(rc, rc)}: {msg}")
    return {k: int(getattr(p, k)) for k in _PLAN_KEYS}


def device_count() -> int:
    L = _lib.load()
    n = ctypes.c_int(0)
    L.hbx_device_count(ctypes.byref(n))
    return int(n.value)


def pack_arena_layout(lens: Sequence[int], align: int = 256):
    """Offsets for packing files into one device arena (16-B aligned, with
    slack after the last file).  Returns (offsets, total_bytes_to_allocate)."""
    offs = np.zeros(len(lens), np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        offs[i] = pos
        pos += (int(n) + align - 1) // align * align
    return offs, pos + max(ARENA_SLACK, align)

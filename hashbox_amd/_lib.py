"""ctypes binding of libhbxgpu.so (the C-ABI declared in include/hbxgpu.h).

There is no fallback: if the library is missing or cannot load, importing the
engine raises.  Build it with ``python -m hashbox_amd.build``.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# The in-tree build only: no environment override, so a variant build can
# never stand in for the product silently (A/B runs copy a variant over this
# file explicitly, tools/gpu_ab.sh).
LIB_PATH = os.path.join(HERE, "libhbxgpu.so")

HBX_OK = 0
ERRORS = {-1: "HBX_ERR_ARG", -2: "HBX_ERR_HIP", -3: "HBX_ERR_CAPACITY", -4: "HBX_ERR_IO",
          -5: "HBX_ERR_NODEV", -6: "HBX_ERR_STATE", -7: "HBX_ERR_FORMAT"}

# Every symbol include/hbxgpu.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "hbx_version", "hbx_device_count", "hbx_max_chunks", "hbx_ctx_create", "hbx_ctx_destroy",
    "hbx_last_error", "hbx_chunk_hash", "hbx_chunk_hash_batch", "hbx_chunk_hash_device",
    "hbx_submit_device", "hbx_wait", "hbx_store_paths", "hbx_block_id", "hbx_md5", "hbx_arena_alloc", "hbx_arena_free",
    "hbx_memcpy_h2d", "hbx_memcpy_h2d_async", "hbx_alloc_pinned", "hbx_free_pinned", "hbx_stage_times",
    "hbx_set_tile_iters", "hbx_pending", "hbx_set_md5_slice", "hbx_stage_totals", "hbx_io_times",
    "hbx_reserve", "hbx_verify_blocks", "hbx_verify_blocks_device",
    "hbx_file_entry_size", "hbx_file_entry_serialize", "hbx_file_entry_parse",
    "hbx_chain_block_serialize", "hbx_chain_block_parse", "hbx_directory_block_size",
    "hbx_directory_block_serialize", "hbx_directory_block_parse", "hbx_directory_block_ids",
    "hbx_deflate_bound", "hbx_deflate_blocks_device", "hbx_deflate_blocks",
    "hbx_deflate_file_bound", "hbx_store_paths_z",
    "hbx_wire_encode_id", "hbx_wire_encode_block_header", "hbx_wire_parse",
    "hbx_verify_submit_device", "hbx_inflate_blocks_device", "hbx_store_paths_zcb", "hbx_after_stream",
    "hbx_set_join_lag", "hbx_set_k3_period", "hbx_k3_wave_times", "hbx_input_after_oldest", "hbx_knobs",
    "hbx_input_fence", "hbx_set_k3_probe", "hbx_store_paths_status", "hbx_plan_pipeline", "hbx_apply_plan",
    "hbx_host_call_max",
]
# Functions returning something other than an int status.
_NON_STATUS = ("hbx_ctx_destroy", "hbx_last_error", "hbx_max_chunks", "hbx_file_entry_size",
               "hbx_directory_block_size", "hbx_deflate_bound", "hbx_deflate_file_bound")


class FileEntry(ctypes.Structure):
    """hbx_file_entry: hashback FileEntry (hashback/hashback.go:80-90)."""
    _fields_ = [("name", ctypes.c_void_p), ("name_len", ctypes.c_uint32), ("file_mode", ctypes.c_uint32),
                ("file_size", ctypes.c_int64), ("mod_time", ctypes.c_int64),
                ("reference_id", ctypes.c_uint8 * 16), ("content_id", ctypes.c_uint8 * 16),
                ("decrypt_key", ctypes.c_uint8 * 16), ("link", ctypes.c_void_p), ("link_len", ctypes.c_uint32),
                ("content_type", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 3)]


class WireMsg(ctypes.Structure):
    """hbx_wire_msg: one parsed protocol message (pkg/core/protocol.go)."""
    _fields_ = [("num", ctypes.c_uint16), ("type", ctypes.c_uint32), ("id", ctypes.c_uint8 * 16),
                ("n_links", ctypes.c_uint32), ("links", ctypes.c_void_p), ("data_type", ctypes.c_uint8),
                ("data_len", ctypes.c_uint32), ("data", ctypes.c_void_p), ("header_len", ctypes.c_uint64),
                ("total_len", ctypes.c_uint64)]


class FileSummary(ctypes.Structure):
    _fields_ = [("content_id", ctypes.c_uint8 * 16), ("content_type", ctypes.c_int32),
                ("n_chunks", ctypes.c_uint32)]


class PlanRequest(ctypes.Structure):
    """hbx_plan_request (include/hbxgpu.h)."""
    _fields_ = [("n_files", ctypes.c_uint64), ("arena_bytes", ctypes.c_uint64), ("longest_file", ctypes.c_uint64),
                ("free_bytes", ctypes.c_uint64), ("hbm_frac", ctypes.c_double),
                ("ranks_per_device", ctypes.c_uint32), ("steps", ctypes.c_uint32), ("arenas", ctypes.c_int32),
                ("md5_slice", ctypes.c_int32), ("join_lag", ctypes.c_int32), ("lead", ctypes.c_int32),
                ("k3_period", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class PipelinePlan(ctypes.Structure):
    """hbx_pipeline_plan (include/hbxgpu.h)."""
    _fields_ = [("resident", ctypes.c_uint32), ("md5_slice", ctypes.c_uint32), ("join_lag", ctypes.c_uint32),
                ("lead", ctypes.c_uint32), ("k3_period", ctypes.c_uint32), ("launches_per_batch", ctypes.c_uint32),
                ("hbm_bytes", ctypes.c_uint64)]


PLAN_HOST_INPUT = 1
PLAN_ARENA_SLACK = 64 << 20

# hbx_batch_ready_fn (include/hbxgpu.h)
BATCH_READY = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64)

_lib = None


def identity() -> dict:
    """Which library this process runs: path and content hash (bench.py
    prints it in its JSON line)."""
    import hashlib
    with open(LIB_PATH, "rb") as fh:
        sha = hashlib.sha256(fh.read()).hexdigest()[:16]
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(HERE)), "sha256_16": sha}


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64
    # (same soname libamdhip64.so.7).  Loading torch first makes our NEEDED
    # entry bind to that copy; loading ours first would put a second HIP/HSA
    # runtime in the process and torch would then see no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m hashbox_amd.build` "
                           "(the engine has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    U64 = ctypes.c_uint64
    I = ctypes.c_int
    L.hbx_version.restype = I
    L.hbx_device_count.argtypes = [ctypes.POINTER(I)]
    L.hbx_max_chunks.argtypes = [U64]
    L.hbx_max_chunks.restype = U64
    L.hbx_ctx_create.argtypes = [I, ctypes.POINTER(P)]
    L.hbx_ctx_destroy.argtypes = [P]
    L.hbx_ctx_destroy.restype = None
    L.hbx_last_error.argtypes = [P]
    L.hbx_last_error.restype = ctypes.c_char_p
    L.hbx_chunk_hash.argtypes = [P, P, U64, P, P, U64, ctypes.POINTER(U64)]
    L.hbx_chunk_hash_batch.argtypes = [P, U64, P, P, P, P, P, P, P]
    L.hbx_chunk_hash_device.argtypes = [P, P, U64, P, P, P, P, P, P, P]
    L.hbx_submit_device.argtypes = [P, P, U64, P, P, P, P, P, P, P]
    L.hbx_wait.argtypes = [P]
    L.hbx_store_paths.argtypes = [P, U64, P, P, P, P, P, P, P, ctypes.c_uint32, U64]
    L.hbx_block_id.argtypes = [P, P, ctypes.c_uint32, P, U64, P]
    L.hbx_md5.argtypes = [P, P, U64, P]
    L.hbx_arena_alloc.argtypes = [P, U64, ctypes.POINTER(P)]
    L.hbx_arena_free.argtypes = [P, P]
    L.hbx_memcpy_h2d.argtypes = [P, P, P, U64]
    L.hbx_memcpy_h2d_async.argtypes = [P, P, P, U64]
    L.hbx_after_stream.argtypes = [P, P]
    L.hbx_alloc_pinned.argtypes = [U64, ctypes.POINTER(P)]
    L.hbx_free_pinned.argtypes = [P]
    L.hbx_stage_times.argtypes = [P, ctypes.POINTER(ctypes.c_float)]
    L.hbx_set_tile_iters.argtypes = [P, ctypes.c_uint32]
    L.hbx_pending.argtypes = [P]
    L.hbx_set_md5_slice.argtypes = [P, ctypes.c_uint32]
    L.hbx_set_join_lag.argtypes = [P, ctypes.c_uint32]
    L.hbx_set_k3_period.argtypes = [P, ctypes.c_uint32]
    L.hbx_input_after_oldest.argtypes = [P]
    L.hbx_input_fence.argtypes = [P, P]
    L.hbx_set_k3_probe.argtypes = [P, I]
    L.hbx_k3_wave_times.argtypes = [P, P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.hbx_knobs.argtypes = [P, ctypes.c_char_p, U64]
    L.hbx_stage_totals.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(U64), I]
    L.hbx_io_times.argtypes = [P, ctypes.POINTER(ctypes.c_double), I]
    L.hbx_host_call_max.argtypes = [P, ctypes.POINTER(ctypes.c_double), I]
    L.hbx_reserve.argtypes = [P, ctypes.c_uint32, U64, U64]
    L.hbx_verify_blocks.argtypes = [P, U64, P, P, P, P, P, P, P, P, ctypes.POINTER(U64)]
    L.hbx_verify_blocks_device.argtypes = [P, P, U64, P, P, P, P, P, P, P, P, ctypes.POINTER(U64)]
    PU64 = ctypes.POINTER(U64)
    PU32 = ctypes.POINTER(ctypes.c_uint32)
    L.hbx_file_entry_size.argtypes = [P]
    L.hbx_file_entry_size.restype = U64
    L.hbx_file_entry_serialize.argtypes = [P, P, U64, PU64]
    L.hbx_file_entry_parse.argtypes = [P, U64, P, PU64]
    L.hbx_chain_block_serialize.argtypes = [P, P, ctypes.c_uint32, P, U64, PU64]
    L.hbx_chain_block_parse.argtypes = [P, U64, PU32, P, P, ctypes.c_uint32]
    L.hbx_directory_block_size.argtypes = [P, ctypes.c_uint32]
    L.hbx_directory_block_size.restype = U64
    L.hbx_directory_block_serialize.argtypes = [P, ctypes.c_uint32, P, U64, PU64, P, PU32]
    L.hbx_directory_block_parse.argtypes = [P, U64, P, ctypes.c_uint32, PU32]
    L.hbx_directory_block_ids.argtypes = [P, ctypes.c_uint32, P, P, P, P]
    L.hbx_deflate_bound.argtypes = [U64]
    L.hbx_deflate_bound.restype = U64
    L.hbx_deflate_blocks_device.argtypes = [P, P, U64, P, P, P, P, P, P]
    L.hbx_deflate_blocks.argtypes = [P, U64, P, P, P, P, P]
    L.hbx_deflate_file_bound.argtypes = [U64]
    L.hbx_deflate_file_bound.restype = U64
    L.hbx_wire_encode_id.argtypes = [ctypes.c_uint16, ctypes.c_uint32, P, P]
    L.hbx_wire_encode_block_header.argtypes = [ctypes.c_uint16, ctypes.c_uint32, P, P, ctypes.c_uint32,
                                               ctypes.c_uint8, ctypes.c_uint32, P, U64, PU64]
    L.hbx_wire_parse.argtypes = [P, U64, P]
    L.hbx_store_paths_zcb.argtypes = [P, U64, P, P, P, P, P, P, P, ctypes.c_uint32, U64, P, P, P, P, P, P]
    L.hbx_inflate_blocks_device.argtypes = [P, P, U64, P, P, P, P, P, P, P]
    L.hbx_verify_submit_device.argtypes = [P, P, U64, P, P, P, P, P, P, P, P, PU64]
    L.hbx_store_paths_z.argtypes = [P, U64, P, P, P, P, P, P, P, ctypes.c_uint32, U64, P, P, P, P]
    L.hbx_store_paths_status.argtypes = [P, U64, P, P, P, P, P, P, P, P, ctypes.c_uint32, U64, P, P, P, P, P, P]
    L.hbx_plan_pipeline.argtypes = [P, ctypes.POINTER(PlanRequest), ctypes.POINTER(PipelinePlan)]
    L.hbx_apply_plan.argtypes = [P, ctypes.POINTER(PipelinePlan), U64, U64]
    for name in EXPORTS:
        if name not in _NON_STATUS:
            getattr(L, name).restype = I
    _lib = L
    return L

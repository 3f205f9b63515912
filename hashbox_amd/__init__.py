"""hashbox_amd — MI355X-native rollsum-split + block-ID engine.

Drop-in for Hashback's chunking hot path (fredli74/hashbox hashback/store.go
storeFile + pkg/core/block.go HashData): hand-written gfx950 HIP kernels behind
the C-ABI in include/hbxgpu.h (libhbxgpu.so), with this package as the host
mirror.  There is no CPU fallback in the product path.
"""
from .engine import (ARENA_ALIGN, ARENA_SLACK, CONTENT_TYPE_FILE_CHAIN, CONTENT_TYPE_FILE_DATA,
                     MAX_BLOCK_SIZE, MIN_BLOCK_SIZE, Engine, FileChunks, HbxError, device_count,
                     max_chunks, pack_arena_layout, plan_pipeline)
from .shard import lpt_assign

__all__ = ["Engine", "FileChunks", "HbxError", "device_count", "max_chunks", "pack_arena_layout",
           "lpt_assign", "plan_pipeline", "MIN_BLOCK_SIZE", "MAX_BLOCK_SIZE", "CONTENT_TYPE_FILE_DATA",
           "CONTENT_TYPE_FILE_CHAIN", "ARENA_ALIGN", "ARENA_SLACK"]

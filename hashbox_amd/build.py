"""Build the native engine in-tree: hashbox_amd/libhbxgpu.so (gfx950 only).

hipcc compiles the kernels (csrc/hbx_kernels.hip) and the host engine + C-ABI
(csrc/hbx_engine.hip, include/hbxgpu.h) into one shared library.  Runs on a
machine without a GPU (cross-compilation).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhbxgpu.so")
SOURCES = ["hbx_engine.hip", "hbx_kernels.hip", "hbx_device.h", "hbx_formats.h", "hbx_deflate.hip", "hbx_inflate.hip", "hbx_inflate_split.hip", "hbx_wire.h",
           os.path.join("..", "..", "include", "hbxgpu.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, s)) > t for s in SOURCES)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           os.path.join(CSRC, "hbx_engine.hip"), "-lhsa-runtime64", "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))

"""Diagnostics: read files from tmpfs into pinned (hbx_alloc_pinned) vs
pageable memory with N threads (os.preadv releases the GIL): is the disk
path's host read bound by the destination memory?"""
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hashbox_amd import _lib  # noqa: E402

d = "/dev/shm/hbx_readdiag"
os.makedirs(d, exist_ok=True)
n, size = 1024, 4 << 20
rng = np.random.default_rng(1)
blob = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
paths = []
for i in range(n):
    p = f"{d}/f{i}"
    if not os.path.exists(p):
        with open(p, "wb") as f:
            f.write(blob)
    paths.append(p)
total = n * size
L = _lib.load()
hp = ctypes.c_void_p()
assert L.hbx_alloc_pinned(total, ctypes.byref(hp)) == 0
pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
pageable = np.empty(total, np.uint8)
pageable[:] = 1  # fault in


def run(buf, threads):
    def one(i):
        fd = os.open(paths[i], os.O_RDONLY)
        mv = memoryview(buf[i * size:(i + 1) * size])
        got = 0
        while got < size:
            got += os.preadv(fd, [mv[got:]], got)
        os.close(fd)
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(n)))
    return total / (time.perf_counter() - t) / 1e9


for th in (1, 4, 16):
    for name, buf in (("pinned", pinned), ("pageable", pageable)):
        run(buf, th)
        print(f"threads={th} {name}: {run(buf, th):.2f} GB/s", flush=True)
t = time.perf_counter()
pageable[:] = pinned
print(f"memcpy pinned->pageable 1 thread: {total / (time.perf_counter() - t) / 1e9:.2f} GB/s")
L.hbx_free_pinned(hp)
for p in paths:
    os.unlink(p)

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
mixed = len(sys.argv) > 1 and sys.argv[1] == "mixed"  # config-5 sizes: log-uniform 4 KiB-4 MiB
n, size = (20000, 4 << 20) if mixed else (1024, 4 << 20)
rng = np.random.default_rng(1)
blob = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
sizes = (np.exp(rng.uniform(np.log(4096), np.log(4 << 20), n)).astype(np.int64) if mixed
         else np.full(n, size, np.int64))
offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
paths = []
for i in range(n):
    p = f"{d}/f{i}"
    if not os.path.exists(p):
        with open(p, "wb") as f:
            f.write(blob[:sizes[i]])
    paths.append(p)
total = int(sizes.sum())
L = _lib.load()
hp = ctypes.c_void_p()
assert L.hbx_alloc_pinned(total, ctypes.byref(hp)) == 0
pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
pageable = np.empty(total, np.uint8)
pageable[:] = 1  # fault in


def run(buf, threads):
    def one(i):
        fd = os.open(paths[i], os.O_RDONLY)
        sz = int(sizes[i])
        mv = memoryview(buf[int(offs[i]):int(offs[i]) + sz])
        got = 0
        while got < sz:
            got += os.preadv(fd, [mv[got:]], got)
        os.close(fd)
    t = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(n)))
    dt = time.perf_counter() - t
    return total / dt / 1e9, n / dt


for th in (1, 4, 16):
    for name, buf in (("pinned", pinned), ("pageable", pageable)):
        run(buf, th)
        gbs, fps = run(buf, th)
        print(f"{'mixed' if mixed else '4MiB'} threads={th} {name}: {gbs:.2f} GB/s, {fps:.0f} files/s", flush=True)
t = time.perf_counter()
pageable[:] = pinned
print(f"memcpy pinned->pageable 1 thread: {total / (time.perf_counter() - t) / 1e9:.2f} GB/s")
L.hbx_free_pinned(hp)
for p in paths:
    os.unlink(p)

"""Diagnostics: the CPU affinity of the calling thread through the stages of a
config-5 run (threads created by the engine inherit the caller's mask), and
the C++ read microbenchmark (tools/ubench/read_files) started from that state."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def show(tag):
    a = sorted(os.sched_getaffinity(0))
    print(f"{tag}: {len(a)} cpus {a[:8]}{'...' if len(a) > 8 else ''}", flush=True)


show("start")
import numpy as np  # noqa: E402,F401
show("numpy")
import torch  # noqa: E402,F401
show("torch")
from hashbox_amd import Engine  # noqa: E402
eng = Engine(0)
show("Engine(0)")
d = "/dev/shm/hbx_aff"
os.makedirs(d, exist_ok=True)
paths = []
for i in range(64):
    p = f"{d}/f{i}"
    with open(p, "wb") as fh:
        fh.write(os.urandom(1 << 20))
    paths.append(p)
eng.store_paths(paths, 16, 64 << 20)
show("store_paths")
try:
    with open("/sys/fs/cgroup/cpu.max") as fh:
        print("cpu.max:", fh.read().strip())
except OSError as e:
    print("cpu.max:", e)
env = dict(os.environ, RD_BIG="1", RD_BATCH="1700")
r = subprocess.run(["tools/ubench/read_files"], env=env, capture_output=True, text=True)
print(r.stdout, r.stderr, flush=True)
eng.close()
for p in paths:
    os.unlink(p)

#!/usr/bin/env python3
"""A whole backup tree end to end (SURVEY §8f1 on top of config 5): 100 k
files (log-uniform 4 KiB-4 MiB, the config-5 distribution) in a 10 x 10 x 10
directory tree on tmpfs, stored with hashbox_amd.formats.store_tree: walk +
Lstat, every file through hbx_store_paths (pipelined K1..K4), then the 1,111
DirectoryBlocks hashed on the device level by level (K6).

Parity: (1) one 1,000-file subtree against the oracle's literal
storePath/storeDir/storeFile recursion (oracle/formats.py); (2) for every
directory of the full tree, id == HashData(dblk, links) on the CPU and the
parent's entry carries the child's id (size-independent properties).

Run on the GPU box: python tools/bench_tree.py [--files 100000]
Prints one JSON line.
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def make_tree(d, n, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    sizes = np.exp(g.uniform(np.log(4096), np.log(4 << 20), n)).astype(np.int64)
    pool = g.integers(0, 256, 512 << 20, dtype=np.uint8)
    offs = g.integers(0, pool.size - (4 << 20), n)
    per_leaf = max(1, n // 1000)
    for i in range(n):
        leaf = i // per_leaf
        sub = os.path.join(d, f"d{leaf // 100 % 10}", f"e{leaf // 10 % 10}", f"f{leaf % 10}")
        os.makedirs(sub, exist_ok=True)
        with open(os.path.join(sub, f"{i:06d}.bin"), "wb") as fh:
            fh.write(pool[offs[i]:offs[i] + sizes[i]].tobytes())
    return int(sizes.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100_000)
    ap.add_argument("--dir", default="/dev/shm/hbx_tree")
    ap.add_argument("--io-threads", type=int, default=16)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process: see hashbox_amd/_lib.py)
    from hashbox_amd import Engine
    from hashbox_amd import formats as F
    from oracle import formats as OF
    from oracle import oracle as O

    shutil.rmtree(a.dir, ignore_errors=True)
    t0 = time.time()
    total = make_tree(a.dir, a.files, 5)
    t_make = time.time() - t0
    root = os.fsencode(a.dir)
    eng = Engine(0)
    try:
        F.store_tree(eng, os.path.join(a.dir, "d0", "e0"), io_threads=a.io_threads)  # warm-up
        eng.io_times(reset=True)
        t0 = time.time()
        got = F.store_tree(eng, a.dir, io_threads=a.io_threads)
        t_all = time.time() - t0
        io = eng.io_times()
        # directory ids alone, all levels in one batch (ids of the children are already final)
        dirs = list(got.directories)
        entries = [F.parse_directory_block(got.directories[p][0]) for p in dirs]
        t0 = time.time()
        ids = F.directory_block_ids(eng, entries)
        t_dirs = time.time() - t0
        ok_props = all(i == got.directories[p][2] == OF.hash_data(got.directories[p][0], got.directories[p][1])
                       for p, i in zip(dirs, ids))
        for p in dirs:
            if p == root:
                continue
            parent = got.directories[os.path.dirname(p)][0]
            ent = [e for e in F.parse_directory_block(parent) if e.file_name == os.path.basename(p)]
            ok_props &= len(ent) == 1 and ent[0].content_block_id == got.directories[p][2]
        sub = os.path.join(root, b"d3", b"e7")
        t0 = time.time()
        want = OF.store_path(sub, O.store_file, toplevel=True)
        t_oracle = time.time() - t0
        sub_bytes = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(sub) for f in fs)
        n_chunks = sum(r.n_chunks for r in got.files.values())
        print(json.dumps({
            "workload": "backup tree: 100k files (config-5 sizes) in 10x10x10 directories, tmpfs, store_tree",
            "files": len(got.files), "directories": len(got.directories), "bytes": total, "chunks": n_chunks,
            "seconds": round(t_all, 3), "gibs": round(total / t_all / 2**30, 3),
            "files_per_s": round(len(got.files) / t_all, 1),
            "phases_s": {k: round(v, 3) for k, v in got.seconds.items()},
            "io_s": {"read": round(io[0], 3), "wait_collect": round(io[1], 3), "wait_copy": round(io[2], 3)},
            "dir_ids_one_batch": {"dirs": len(dirs), "ms": round(t_dirs * 1e3, 3),
                                  "dblk_bytes": sum(len(got.directories[p][0]) for p in dirs)},
            "root_id": got.root.content_block_id.hex(),
            "parity_subtree_vs_oracle": want.content_id == got.directories[sub][2],
            "oracle_subtree": {"bytes": sub_bytes, "seconds": round(t_oracle, 3),
                               "gibs_1core": round(sub_bytes / t_oracle / 2**30, 3)},
            "parity_all_dirs_properties": bool(ok_props),
            "make_s": round(t_make, 1),
        }), flush=True)
    finally:
        eng.close()
        if not a.keep:
            shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()

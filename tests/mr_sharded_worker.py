"""One rank of tests/test_gpu_multirank.py (launched by torch.distributed.run
before any GPU call): files sharded by LPT across the ranks
(hashbox_amd.multi.run_sharded), each rank chunks + hashes its shard on the
GPU through the pipelined engine (submit / wait), results all-gathered over
gloo; rank 0 checks every file against the oracle and prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SIZES = [3_000_000, 17, 0, 9_000_001, 131_073, 2_500_000, 6_000_000, 700_000, 12_345_678, 65_536, 40_000_000]


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from hashbox_amd import Engine, pack_arena_layout
    from hashbox_amd.multi import run_sharded
    from oracle import oracle as O
    files = [O.random_bytes(n, 900 + i) for i, n in enumerate(SIZES)]
    files[4] = np.full(SIZES[4], 0x5A, np.uint8)

    def process(idx):
        eng = Engine(0, md5_slice=int(os.environ.get("MR_SLICE", "2048")))
        lens = [SIZES[i] for i in idx]
        offs, total = pack_arena_layout(lens)
        host = np.zeros(total, np.uint8)
        for o, i in zip(offs, idx):
            host[int(o):int(o) + SIZES[i]] = files[i]
        dev = torch.from_numpy(host).to("cuda:0")
        out = {}
        half = len(idx) // 2  # two batches in flight on this rank's context
        parts = [(idx[:half], offs[:half], lens[:half]), (idx[half:], offs[half:], lens[half:])]
        for _, o, n in parts:
            eng.submit_device(dev.data_ptr(), o, n)
        for ids_, _, _ in parts:
            for i, r in zip(ids_, eng.wait()):
                out[i] = (r.cut_ends.tolist(), [bytes(x).hex() for x in r.ids], r.content_type, r.content_id.hex())
        eng.close()
        return out

    res = run_sharded(SIZES, process, rank, world)
    if rank == 0:
        ok = sorted(res) == list(range(len(SIZES)))
        for i, f in enumerate(files):
            r = O.store_file(f, fast=True)
            ok = ok and res[i][0] == r.cut_ends.tolist() and res[i][1] == [bytes(x).hex() for x in r.ids]
            ok = ok and res[i][2] == r.content_type and res[i][3] == r.content_id.hex()
        print(json.dumps({"ok": bool(ok), "files": len(res), "world": world}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

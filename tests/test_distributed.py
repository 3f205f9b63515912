"""CPU, world_size 2 over gloo: the N>1 path shards files by LPT, processes
each shard independently (here with the CPU oracle standing in for the
device) and gathers results; the union must equal the single-process run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _files():
    from oracle import oracle as O
    sizes = [3_000_000, 17, 0, 9_000_001, 131_073, 2_500_000, 6_000_000, 700_000]
    return [O.random_bytes(n, 500 + i) for i, n in enumerate(sizes)]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hashbox_amd.multi import max_over_ranks, run_sharded
    from oracle import oracle as O
    files = _files()

    def process(idx):
        return {i: (O.store_file(files[i], fast=True).cut_ends.tolist(),
                    [bytes(x).hex() for x in O.store_file(files[i], fast=True).ids]) for i in idx}

    res = run_sharded([f.size for f in files], process, rank, world)
    t = max_over_ranks(0.5 + rank)
    if rank == 0:
        q.put((res, t))
    dist.barrier()
    dist.destroy_process_group()


def test_lpt_balance():
    from hashbox_amd.shard import lpt_assign
    lens = [100, 90, 80, 70, 60, 50, 40, 30]
    parts = lpt_assign(lens, 3)
    assert sorted(sum(parts, [])) == list(range(8))
    loads = [sum(lens[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= 40


def test_gloo_world2_sharded_matches_single():
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == pytest.approx(1.5)
    files = _files()
    assert sorted(res) == list(range(len(files)))
    for i, f in enumerate(files):
        r = O.store_file(f, fast=True)
        assert res[i][0] == r.cut_ends.tolist()
        assert res[i][1] == [bytes(x).hex() for x in r.ids]

#!/usr/bin/env python3
"""Benchmark: device-resident rollsum split + block-ID hashing on MI355X.

Workload (BASELINE.json configs[1]): 64 x 128 MiB uniform random buffers per
GPU, resident in HBM before the timed region.  One step = one pass of the hot
path over that batch: K1 window-digest scan -> K2 cut chain -> K3 block MD5 ->
K4 content ids -> D2H of cut lists + block IDs.  Files shard by GPU (weak
scaling: each rank owns its own 64-file batch, no collective on the data path;
the only collectives are the start/end barrier and the max-time reduction).

Prints ONE JSON line on rank 0.  Multi-GPU:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "device-resident GiB/s chunked+hashed at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md), GB/s
GIB = 1 << 30


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--file-mib", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-files", type=int, default=32,
                    help="files of the batch timed on the CPU oracle (bounded sample)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="batches in flight (one engine context + one resident batch each); "
                         "1 = every step runs alone")
    ap.add_argument("--e2e", action="store_true",
                    help="host-inclusive mode: files in pinned host memory, H2D of batch i+1 "
                         "overlapped with the kernels of batch i (two contexts)")
    ap.add_argument("--check", action="store_true",
                    help="verify the first file of the batch against the oracle")
    return ap.parse_args()


def cpu_baseline(host_files, threads):
    """Oracle ('port': the literal store.go:111-185 loop + RFC 1321 MD5) on the
    host cores, on a bounded sample of the same batch."""
    from oracle import oracle as O
    O.lib()
    nbytes = sum(int(f.size) for f in host_files)
    t0 = time.perf_counter()
    O.store_batch_mt(host_files, threads)
    t_mt = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.store_file(host_files[0])
    t_1 = time.perf_counter() - t0
    return {
        "value": round(nbytes / t_mt / GIB, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{len(host_files)} of the batch's 128 MiB files ({nbytes / GIB:.1f} GiB), "
                  f"one file per thread, literal storeFile loop + MD5 (oracle/hbx_oracle.c)",
        "single_core_gibs": round(host_files[0].size / t_1 / GIB, 4),
        "seconds": round(t_mt, 2),
    }


def run_e2e(a, local):
    """PCIe-inclusive rate: the batch starts in pinned host memory and its
    results end in host memory.  Two engine contexts alternate so the H2D
    copy of batch i+1 (DMA engine) overlaps the kernels of batch i."""
    import ctypes
    from hashbox_amd import Engine, pack_arena_layout
    nf, fbytes = a.files, a.file_mib << 20
    lens = [fbytes] * nf
    offs, total = pack_arena_layout(lens)
    engs = [Engine(local), Engine(local)]
    arenas = [torch.empty(total, dtype=torch.uint8, device=f"cuda:{local}") for _ in range(2)]
    hp = ctypes.c_void_p()
    assert engs[0]._L.hbx_alloc_pinned(total, ctypes.byref(hp)) == 0
    host = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(hp.value))
    g = torch.Generator(device=f"cuda:{local}")
    g.manual_seed(a.seed)
    arenas[0].random_(0, 256, generator=g)
    host[:] = arenas[0].cpu().numpy()

    def one(i):
        e, d = engs[i % 2], arenas[i % 2]
        e.memcpy_h2d_async(d.data_ptr(), hp.value, total)
        e.submit_device(d.data_ptr(), offs, lens)

    res = None
    for i in range(a.warmup):  # untimed, each batch completed
        one(i)
        res = engs[i % 2].wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(a.steps):  # batch j's copy+kernels overlap batch j-1's
        one(j)
        if j > 0:
            res = engs[(j - 1) % 2].wait()
    res = engs[(a.steps - 1) % 2].wait()
    el = time.perf_counter() - t0
    gib = a.steps * nf * fbytes / el / GIB
    out = {"metric": "end-to-end GiB/s, pinned host memory -> HBM -> chunk lists + block IDs in "
                     "host memory (H2D overlapped with kernels)",
           "value": round(gib, 3), "unit": "GiB/s", "n_gpus": 1, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
           "config": {"workload": f"{nf} x {a.file_mib} MiB random buffers", "contexts": 2},
           "chunks_per_step": sum(r.n_chunks for r in res)}
    print(json.dumps(out), flush=True)
    for e in engs:
        e.close()
    engs[0]._L.hbx_free_pinned(hp)


def main():
    a = parse()
    if a.e2e:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        return run_e2e(a, int(os.environ.get("LOCAL_RANK", "0")))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if rank == 0:
            print(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
                  file=sys.stderr)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from hashbox_amd import Engine, pack_arena_layout

    dev = torch.device("cuda", local)
    nf, fbytes = a.files, a.file_mib << 20
    lens = [fbytes] * nf
    offs, total = pack_arena_layout(lens)
    D = max(1, a.inflight)
    # synthetic uniform random bytes, generated on the device (per-rank seed);
    # one resident batch per in-flight context
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed + 7919 * rank)
    arenas = []
    for _ in range(D):
        t = torch.empty(total, dtype=torch.uint8, device=dev)
        t.random_(0, 256, generator=g)
        arenas.append(t)
    arena = arenas[0]
    torch.cuda.synchronize()

    engs = [Engine(local) for _ in range(D)]
    eng = engs[0]

    res = None
    for i in range(a.warmup):
        engs[i % D].submit_device(arenas[i % D].data_ptr(), offs, lens)
        res = engs[i % D].wait()

    stage = np.zeros(5)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    results = {}
    for j in range(a.steps):
        e = engs[j % D]
        if j >= D:  # this context's previous batch must be collected first
            results[j - D] = e.wait()
            stage += e.stage_times()
        e.submit_device(arenas[j % D].data_ptr(), offs, lens)
    for j in range(max(0, a.steps - D), a.steps):
        e = engs[j % D]
        results[j] = e.wait()
        stage += e.stage_times()
    res = results[a.steps - 1] if a.steps else res
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    el = t1 - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    stage /= max(a.steps, 1)
    n_chunks = sum(r.n_chunks for r in res)
    longest = max(int(np.max(np.diff(np.concatenate([[0], r.cut_ends]).astype(np.int64))))
                  for r in res if r.n_chunks)

    check = None
    if a.check and rank == 0:
        from oracle import oracle as O
        h0 = arenas[(a.steps - 1) % D][int(offs[0]):int(offs[0]) + fbytes].cpu().numpy()
        ref = O.store_file(h0, fast=True)
        check = bool(np.array_equal(ref.cut_ends, res[0].cut_ends)
                     and np.array_equal(ref.ids, res[0].ids))

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        k = min(a.cpu_files, nf)
        host = [arena[int(offs[i]):int(offs[i]) + fbytes].cpu().numpy() for i in range(k)]
        cpu = cpu_baseline(host, a.cpu_threads)
        del host

    batch_bytes = nf * fbytes
    total_bytes = batch_bytes * world * a.steps
    value = total_bytes / el / GIB
    names = ["k1_digest_scan", "k2_cut_chain", "k3_block_md5", "k4_content_id"]
    dom = int(np.argmax(stage[:4]))
    achieved = batch_bytes / (stage[dom] * 1e-3) / 1e9  # GB/s, algorithmic bytes = input bytes
    k1_gbs = batch_bytes / (stage[0] * 1e-3) / 1e9 if stage[0] > 0 else 0.0
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: uniform random bytes generated on the device (torch Generator), "
                "resident in HBM before timing",
        "config": {"workload": f"{nf} x {a.file_mib} MiB random buffers per GPU, rollsum split + "
                               "MD5 block IDs + file content ids, device-resident (configs[1])",
                   "files_per_gpu": nf, "file_bytes": fbytes, "chunks_per_gpu": n_chunks,
                   "longest_chunk_bytes": longest,
                   "parallelism": f"file-sharded x{world} (independent HIP streams, no data-path "
                                  "collective)",
                   "batches_in_flight": D},
        "roofline": {"kernel": names[dom], "bound": "hbm", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": None},
        "stages_ms": {n: round(float(v), 4) for n, v in zip(names + ["batch"], stage)},
        "k1_roofline": {"achieved": round(k1_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(k1_gbs / HBM_PEAK_GBS, 4)},
        "cpu_baseline": cpu,
    }
    if check is not None:
        out["check_vs_oracle"] = check
    if rank == 0:
        print(json.dumps(out), flush=True)
    for e in engs:
        e.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

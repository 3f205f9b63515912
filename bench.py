#!/usr/bin/env python3
"""Benchmark: device-resident rollsum split + block-ID hashing on MI355X.

Workload (BASELINE.json configs[1]): batches of 64 x 128 MiB uniform random
buffers per GPU, resident in HBM before the timed region.  One step = one
batch through the whole hot path: K1 window-digest scan -> K2 cut chain ->
K3 block MD5 -> K4 content ids -> D2H of cut lists + block IDs.  Steps
pipeline on one engine context: K3 is time-sliced (--md5-slice blocks per
chain per launch), so each step's chunks join the MD5 chains still in flight
and no batch waits behind another's longest chunk.  The timed region runs K
steps from an empty pipeline to a fully drained one (every batch's results
collected); `value` = K batches / that time.  --md5-slice 0 runs every batch
alone (one K3 launch per batch: the single-batch latency path).  Files shard
by GPU (weak scaling: each rank owns its own batches, no collective on the
data path; the only collectives are the start/end barrier and the max-time
reduction).

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
K3_VALU_PER_BLOCK = 325
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md), GB/s
GIB = 1 << 30


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--file-mib", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-files", type=int, default=32,
                    help="files of the batch timed on the CPU oracle (bounded sample)")
    ap.add_argument("--md5-slice", type=int, default=-1,
                    help="K3 time slice in 64-B MD5 blocks per chain per launch (0 = each batch "
                         "hashed alone in one launch; -1 = sized from HBM, see --hbm-frac)")
    ap.add_argument("--arenas", type=int, default=0,
                    help="distinct resident batches (default: the pipeline depth the slice "
                         "schedule needs, so no step forces a drain)")
    ap.add_argument("--hbm-frac", type=float, default=0.95,
                    help="with --md5-slice -1: fraction of free HBM given to resident batches; "
                         "throughput ~ resident bytes / batch latency (the longest chunk's "
                         "serial MD5), so the pipeline is made as deep as this allows")
    ap.add_argument("--lead", type=int, default=2,
                    help="steps the scan stream (K1/K2 of a new batch) may run ahead of the hash "
                         "stream: the pipeline holds launches-per-batch + lead batches")
    ap.add_argument("--e2e", action="store_true",
                    help="host-inclusive mode: files in pinned host memory, H2D of batch i+1 "
                         "overlapped with the kernels of batch i (two contexts)")
    ap.add_argument("--check", action="store_true",
                    help="verify the first file of the batch against the oracle")
    return ap.parse_args()


def measured_traffic(kernel, nf, fbytes):
    """HBM bytes per launch of `kernel` from the newest committed PMC pass of
    this same workload (profiles/*_traffic.json, written by
    tools/pmc_traffic.py from a separate rocprofv3 --pmc FETCH_SIZE run: PMC
    counters cannot be read inside this timed run)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    if not files or (nf, fbytes) != (64, 128 << 20):  # measured on the default workload only
        return None, None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return int(k["hbm_bytes"]), (os.path.relpath(files[-1], ROOT) +
                                 ("" if k.get("calibrated") else " (uncalibrated access width)"))


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
    engs = [Engine(local, md5_slice=0), Engine(local, md5_slice=0)]
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
    # launches a batch needs before its chains are all hashed; a batch can be
    # collected without a forced drain once `need` newer steps have launched
    nfull = (min(fbytes, 8 << 20) + 8) >> 6
    # a batch holds its arena from its K1 until its last K3 launch; with
    # `lead` more arenas than launches per batch, the scan stream runs `lead`
    # steps ahead of the hash stream and never waits for a collect
    free, _ = torch.cuda.mem_get_info(dev)
    r_fit = max(a.lead + 1, int(free * a.hbm_frac) // (total + (64 << 20)))
    if a.md5_slice < 0:
        R = a.arenas if a.arenas > 0 else r_fit
        B = -(-nfull // max(1, R - a.lead))
    else:
        B = a.md5_slice
    need = 1 if B == 0 else -(-nfull // B)
    if a.arenas > 0:
        R = a.arenas
    elif a.md5_slice >= 0:
        # a short slice needs more launches per batch than HBM holds batches:
        # cap the residency (collects then wait for the hash stream)
        R = min(need + a.lead, r_fit)
    # synthetic uniform random bytes, generated on the device (per-rank seed);
    # R distinct resident batches, batch j reads arena j % R
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed + 7919 * rank)
    arenas = []
    for _ in range(R):
        t = torch.empty(total, dtype=torch.uint8, device=dev)
        t.random_(0, 256, generator=g)
        arenas.append(t)
    arena = arenas[0]
    torch.cuda.synchronize()

    eng = Engine(local, md5_slice=B)
    # every batch slot, chain table and summary buffer of the pipeline is
    # allocated now: an allocation inside the timed region would drain both
    # streams
    eng.reserve(R + 1, nf, nf * fbytes)
    # single-batch latency (one batch alone, synchronous call), untimed
    for _ in range(2):
        eng.chunk_hash_device(arena.data_ptr(), offs, lens)
    latency = eng.stage_times()

    def run(steps):
        """steps batches through the pipeline, fully drained; last result."""
        last = None
        for j in range(steps):
            if eng.pending() >= R:  # arena j % R is free once its batch is collected
                last = eng.wait()
            eng.submit_device(arenas[j % R].data_ptr(), offs, lens)
        while eng.pending():
            last = eng.wait()
        return last

    run(a.warmup)
    eng.stage_totals(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = run(a.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    el = t1 - t0
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    tot_ms, tot_n = eng.stage_totals()
    n_chunks = sum(r.n_chunks for r in res)
    longest = max(int(np.max(np.diff(np.concatenate([[0], r.cut_ends]).astype(np.int64))))
                  for r in res if r.n_chunks)

    check = None
    if a.check and rank == 0:  # every file of the last timed batch vs the oracle
        from oracle import oracle as O
        last = arenas[(a.steps - 1) % R]
        host = [last[int(o):int(o) + fbytes].cpu().numpy() for o in offs]
        refs = O.store_batch_mt(host, a.cpu_threads)
        check = all(np.array_equal(r.cut_ends, g.cut_ends) and np.array_equal(r.ids, g.ids)
                    for r, g in zip(refs, res)) and len(res) == len(refs)
        del host

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        k = min(a.cpu_files, nf)
        host = [arena[int(offs[i]):int(offs[i]) + fbytes].cpu().numpy() for i in range(k)]
        cpu = cpu_baseline(host, a.cpu_threads)
        del host

    batch_bytes = nf * fbytes
    total_bytes = batch_bytes * world * a.steps
    value = total_bytes / el / GIB
    names = ["k1_digest_scan", "k2_cut_chain", "k2c_chain_plan", "k3_block_md5", "k4_content_id"]
    kernel_of = {"k1_digest_scan": "hbx_k1_digest_scan_dma", "k2_cut_chain": "hbx_k2_cut_chain",
                 "k2c_chain_plan": "hbx_k2c_plan", "k3_block_md5": "hbx_k3_block_md5",
                 "k4_content_id": "hbx_k4_content_id"}
    avg_ms = tot_ms / np.maximum(tot_n, 1)
    dom = int(np.argmax(tot_ms))
    # algorithmic bytes per launch: every input byte is scanned once by K1 and
    # MD5-hashed once by K3, so a kernel's average launch covers
    # (bytes of the K batches) / (its launches); K2/K2c/K4 are priced the same
    per_launch = a.steps * batch_bytes / max(int(tot_n[dom]), 1)
    achieved = per_launch / (avg_ms[dom] * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic(kernel_of[names[dom]], nf, fbytes)
    k1_gbs = (a.steps * batch_bytes / max(int(tot_n[0]), 1)) / (avg_ms[0] * 1e-3) / 1e9 \
        if tot_ms[0] > 0 else 0.0
    k3_bps = a.steps * batch_bytes / (tot_ms[3] * 1e-3) if tot_ms[3] > 0 else 0.0
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
        "data": f"synthetic: uniform random bytes generated on the device (torch Generator), "
                f"{R} distinct resident batches, resident in HBM before timing",
        "config": {"workload": f"{nf} x {a.file_mib} MiB random buffers per GPU per step, rollsum "
                               "split + MD5 block IDs + file content ids, device-resident "
                               "(configs[1])",
                   "files_per_step": nf, "file_bytes": fbytes, "chunks_per_step": n_chunks,
                   "longest_chunk_bytes": longest, "md5_slice_blocks": B,
                   "pipeline_depth": R, "launches_per_batch": need, "scan_lead": a.lead,
                   "k1_kernel": os.environ.get("HBX_K1_MODE", "default"),
                   "parallelism": f"file-sharded x{world} (independent HIP streams, no data-path "
                                  "collective)"},
        "roofline": {"kernel": names[dom], "bound": "hbm", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "launches": int(tot_n[dom]), "avg_launch_ms": round(float(avg_ms[dom]), 4),
                     "algorithmic_bytes_per_launch": int(per_launch)},
        # K3 is VALU-issue work: ~325 VALU per 64-B block on the cooperative path
        # (5 per MD5 step).  Chip peak = 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz;
        # one wave alone issues at most one VALU per 4 cycles (MI355X_MICROARCH.md),
        # so one serial chain is floored at 325 x 4 cycles per block.
        "k3_valu": {"valu_per_block": K3_VALU_PER_BLOCK,
                    "achieved_tops": round(k3_bps * K3_VALU_PER_BLOCK / 64 / 1e12, 3),
                    "peak_tops": round(VALU_PEAK_LANE_OPS / 1e12, 2),
                    "frac": round(k3_bps * K3_VALU_PER_BLOCK / 64 / VALU_PEAK_LANE_OPS, 4)},
        "kernel_ms_per_step": {n: round(float(v) / a.steps, 4) for n, v in zip(names, tot_ms)},
        "kernel_launches": {n: int(v) for n, v in zip(names, tot_n)},
        "k1_roofline": {"achieved": round(k1_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(k1_gbs / HBM_PEAK_GBS, 4)},
        "single_batch": {"ms": round(float(latency[4]), 3),
                         "gibs": round(batch_bytes / GIB / (float(latency[4]) * 1e-3), 3),
                         "stages_ms": [round(float(x), 3) for x in latency]},
        "cpu_baseline": cpu,
    }
    if check is not None:
        out["check_vs_oracle"] = check
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

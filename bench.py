#!/usr/bin/env python3
"""Benchmark: device-resident rollsum split + block-ID hashing on MI355X.

Workload (BASELINE.json configs[1]): a step is one batch of 64 x 128 MiB
uniform random buffers (8 GiB) through the whole hot path: K1 window-digest
scan -> K2 cut chain -> K3 block MD5 -> K4 content ids -> D2H of cut lists +
block IDs (hashback/store.go:111-196, pkg/core/block.go:96-111).  Inputs are
resident in HBM before timing.

Steady state.  Steps pipeline on one engine context: K3 is time-sliced
(--md5-slice blocks per chain per launch), so each batch's chunks join the
MD5 chains still in flight.  Before the timer the pipeline is filled to its
operating depth (R batches submitted, none collected) and run W warm-up
steps.  The timed region is exactly K steps; a step collects the oldest
batch (already complete: every chain hashed, results in host memory) and
submits one new batch, i.e. one K1 and one K3 launch per step (asserted from
the engine's own launch counts).  The drain that empties the pipeline runs
after the timer and is reported beside `value` (`drain_ms`,
`fill_drain_gibs` = the whole run from an empty pipeline to a drained one).

Multi-GPU (--scaling strong, the default: BASELINE configs[2]): every step's
64 x 128 MiB files are split across the ranks by LPT on bytes
(hashbox_amd.shard), each rank pipelines its share on its own GPU and
streams; value = 8 GiB x K / the slowest rank's time.  --scaling weak (opt
in): every rank takes a whole batch of its own files per step (configs[1] per
GPU); value = N x 8 GiB x K / the slowest rank's time.  No collective touches
the data: torch.distributed carries only the barriers, the max-time reduction
and the check flags.

End to end (key `e2e`, on by default, --e2e-steps 0 turns it off): after the
device-resident lines, the same pipeline with every step's batch copied from
pinned host memory (hbx_alloc_pinned + hbx_memcpy_h2d_async on the scan
stream, overlapped with the previous batches' kernels), results back in host
memory: the PCIe-inclusive rate north_star asks for (store.go:125 fill,
client.go:249-258 send).

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
from collections import deque

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "device-resident GiB/s chunked+hashed at 1/2/4/8 MI355X; % HBM roofline"
K3_VALU_PER_BLOCK = 325
# VALU issue ceiling (DESIGN.md §6 "The bound"), measured by
# tools/ubench/valu_issue.hip on every SIMD of the chip with every wave
# stamped (profiles/r03b/valu_issue.txt, r03d, r03f):
#  * half-rate ops (v_add3, v_alignbit, SDWA, DPP, v_max3, v_perm, v_dot4,
#    v_lshl_add, v_lshlrev, v_max_u32, ...): 4.10 cycles per wave64
#    instruction per SIMD at 8 waves per SIMD, never dual-issued;
#  * full-rate ops (v_add_u32, v_xor/and/or, v_bitop3, v_lshrrev, 16-bit
#    VOP2 adds, v_fma_f32): 2.2-2.5 cycles with >= 2 waves (two waves
#    dual-issue, SQ_ACTIVE_INST_VALU2), 4.66 with one wave;
#  * one wave alone issues at most one instruction per ~4.1 cycles whatever
#    its class (the compiler's MD5 step chain: 21.1 cycles per 5.1 VALU).
# K1's scan is all half-rate ops at four waves per SIMD, and K3 runs one wave
# per SIMD (a chain's speed, not the SIMD's total rate, sets the pipeline's
# throughput at fixed residency: DESIGN.md §6), so both are capped at one
# wave64 VALU per 4.10 cycles per SIMD.  Per-byte instruction counts: PMC
# SQ_INSTS_VALU per launch of the default workload (profiles/r03c).
K1_WAVE_VALU_PER_BYTE = 6.825e8 / (8 << 30)
K3_WAVE_VALU_PER_BYTE = 6.901e8 / (8 << 30)
SIMD_CYCLES_PER_VALU = 4.10
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / SIMD_CYCLES_PER_VALU
VALU_SOURCE = "tools/ubench/valu_issue.hip (profiles/r03b/valu_issue.txt); SQ_INSTS_VALU profiles/r03c"
# Achievable HBM read bandwidth (tools/ubench/roofline_probe, round 1), and
# the path's two reads of every byte: K1 scans it, K3 hashes it once its cut
# is known (the first MD5 block holds BE32(len)), so the algorithmic rate is
# at most half of what HBM delivers.
HBM_PROBE_GBS = 6580.0
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md), GB/s
GIB = 1 << 30
KNAMES = ["k1_digest_scan", "k2_cut_chain", "k2c_chain_plan", "k3_block_md5", "k4_content_id"]
KERNEL_OF = {"k1_digest_scan": ("hbx_k1d_digest_scan", "hbx_k1_digest_scan_dma"), "k2_cut_chain": "hbx_k2_cut_chain",
             "k2c_chain_plan": "hbx_k2c_plan", "k3_block_md5": "hbx_k3p_block_md5",  # K3P, the default since round 5
             "k4_content_id": "hbx_k4_content_id"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--files", type=int, default=64, help="files per step (whole job)")
    ap.add_argument("--file-mib", type=int, default=128)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong (default, configs[2]): each step's files are split across the ranks; "
                         "weak: every rank takes a whole batch of its own files per step (per-GPU work fixed)")
    ap.add_argument("--workload", choices=["both", "random", "zipf"], default="both",
                    help="both: the random headline plus a Zipf-duplicate line under key 'zipf'")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--cpu-files", type=int, default=64,
                    help="files of the batch timed on the CPU oracle (bounded sample)")
    ap.add_argument("--md5-slice", type=int, default=-1,
                    help="K3 time slice in 64-B MD5 blocks per chain per launch (-1 = sized from "
                         "the residency: ceil(blocks of an 8 MiB chunk / (R - lead)))")
    ap.add_argument("--arenas", type=int, default=0,
                    help="distinct resident batches R (default: as many as --hbm-frac of free HBM holds)")
    ap.add_argument("--hbm-frac", type=float, default=0.95,
                    help="fraction of free HBM given to resident batches; throughput ~ resident bytes "
                         "/ batch lifetime (the longest chunk's serial MD5)")
    ap.add_argument("--join-lag", type=int, default=0,
                    help="submits between a batch's own and the K3 launch its chains join "
                         "(hbx_set_join_lag; 0 = auto: 2)")
    ap.add_argument("--k3-period", type=int, default=0,
                    help="one K3 launch every P submits with P x the slice (hbx_set_k3_period, 1..8; 0 = auto: "
                         "1 at 32 or more files per GPU, else 4 (or 2) if it divides --steps)")
    ap.add_argument("--lead", type=int, default=-1,
                    help="steps an arena stays resident beyond the launches its batch needs: R = launches "
                         "per batch + lead (-1 = the library's: the join lag at 64+ files per GPU, lag + 1 below "
                         "and with --e2e).  Lead = join lag is the least that lets the next batch's scan overlap "
                         "the launch finishing the old one (hbx_input_after_oldest)")
    ap.add_argument("--e2e", action="store_true",
                    help="host-inclusive mode as the headline: each step's batch is copied from pinned host "
                         "memory (H2D on the engine's scan stream, overlapped with the pipeline)")
    ap.add_argument("--e2e-steps", type=int, default=20,
                    help="steps of the pinned-host leg reported under key 'e2e' after the device-resident "
                         "lines (0 = skip)")
    ap.add_argument("--no-lifetime", action="store_true",
                    help="skip the probed lifetime decomposition after the timed window (key 'lifetime')")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the oracle check of the last collected and the last drained batch")
    ap.add_argument("--check-batches", type=int, default=1,
                    help="batches collected in the timed window checked file by file against the oracle "
                         "(the last K, each its own arena; default 1), besides the last drained one")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on GPUs; gloo for tests")
    ap.add_argument("--dist-always", action="store_true",
                    help="join a process group even at world 1 (exercises the RCCL barriers and reductions "
                         "on a one-GPU box)")
    ap.add_argument("--ballast-gib", type=float, default=0.0,
                    help="diagnostics: hold this much extra device memory (written once, never read)")
    ap.add_argument("--k3-probe", action="store_true",
                    help="diagnostics: per-wave timeline of the window's last K3 launch (hbx_set_k3_probe)")
    ap.add_argument("--alias-depth", type=int, default=0,
                    help="diagnostics: D batches in flight over the physical arenas (batch j reads arena "
                         "j %% R; inputs are read-only, so aliasing emulates the residency a paged arena would "
                         "free).  Never the headline: the line is marked 'aliased'")
    ap.add_argument("--single-alloc", action="store_true",
                    help="the R arenas as views of one allocation instead of R allocations")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds a rank waits in torch.distributed setup and collectives before failing")
    ap.add_argument("--plan-only", action="store_true",
                    help="print each rank's residency plan (no GPU work) and exit; with --free-gib it runs "
                         "on a CPU host (tests)")
    ap.add_argument("--free-gib", type=float, default=0.0,
                    help="--plan-only: free HBM per device to plan for (default: the device's)")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="diagnostics: this rank raises during setup (every rank must then exit non-zero)")
    return ap.parse_args()


# ------------------------------------------------------------------ host --
def cpu_info():
    """Cores this process may use (affinity and cgroup quota) and the model."""
    n_os = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = n_os
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"os_cpu_count": n_os, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable,
            "model": model}


def cpu_baseline(host_files, threads, info):
    """Oracle ('port': oracle/hbx_oracle.c, the C restatement of the literal
    storeFile loop store.go:111-185 + MD5 framing block.go:96-111, standing
    in for the Go reference: the image has no Go toolchain) on the host
    cores, on a bounded sample of the same batch."""
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
        "sample": f"{len(host_files)} of the batch's {host_files[0].size >> 20} MiB files "
                  f"({nbytes / GIB:.1f} GiB), files spread over {threads} threads",
        "what": "oracle/hbx_oracle.c: C restatement of store.go:111-185 + block.go:96-111 "
                "(stands in for the Go reference, which cannot be built here)",
        "single_core_gibs": round(host_files[0].size / t_1 / GIB, 4),
        "seconds": round(t_mt, 2), "cpu": info,
    }


def oracle_check(arena, offs, lens, res, threads):
    """Every file of one collected batch against the oracle (outside the timer)."""
    from oracle import oracle as O
    used = int(offs[-1]) + int(lens[-1])
    host = arena[:used].cpu().numpy()
    files = [host[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
    refs = O.store_batch_mt(files, threads)
    ok = len(refs) == len(res)
    for r, g in zip(refs, res):
        ok = ok and np.array_equal(r.cut_ends, g.cut_ends) and np.array_equal(r.ids, g.ids)
    return bool(ok)


TRAFFIC_FILE = "profiles/r06zd_traffic.json"  # PMC FETCH_SIZE pass of the round-6 final kernels (tools/profile_round.sh)


def measured_traffic(kernel, per_launch_bytes, batch_bytes):
    """HBM bytes per launch of `kernel` from the newest committed PMC pass of
    the default workload (profiles/*_traffic.json, tools/pmc_traffic.py from a
    separate rocprofv3 --pmc FETCH_SIZE run: PMC counters cannot be read
    inside this timed run), scaled to this launch's bytes."""
    import glob
    # the round's final profile by name (round tags do not sort by date:
    # r03f is round 3's final tree, after r03z), else the last by name
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    pick = os.path.join(ROOT, TRAFFIC_FILE)
    if os.path.exists(pick):
        files.append(pick)
    if not files or batch_bytes != 64 * (128 << 20):
        return None, None
    d = json.load(open(files[-1]))
    kk = d.get("kernels", {})
    # K1 may be named by more than one kernel (older profiles name K1D, the pruned round-6 variant)
    k = next((kk[n] for n in ((kernel,) if isinstance(kernel, str) else kernel) if n in kk), None)
    if not k:
        return None, None
    return int(k["hbm_bytes"]), os.path.relpath(files[-1], ROOT)


def path_roofline(alg_bps, batch_bytes):
    """Every byte is read twice per step (K1, then K3), so the algorithmic
    rate can reach at most half of the HBM read bandwidth: with the probe's
    6.58 TB/s that is 3.29 TB/s, 41 % of the 8 TB/s spec, for any design that
    hashes after cutting.  `read_bytes_per_step` is the measured traffic of
    both kernels (PMC FETCH_SIZE, tools/pmc_traffic.py)."""
    t1, src = measured_traffic(KERNEL_OF["k1_digest_scan"], batch_bytes, batch_bytes)
    t3, _ = measured_traffic(KERNEL_OF["k3_block_md5"], batch_bytes, batch_bytes)
    alg = alg_bps / 1e9
    out = {"unit": "GB/s", "algorithmic": round(alg, 2), "peak": HBM_PEAK_GBS,
           "reads_per_byte": 2, "two_read_ceiling": round(HBM_PROBE_GBS / 2, 1),
           "frac_of_two_read_ceiling": round(alg / (HBM_PROBE_GBS / 2), 4),
           "two_read_ceiling_frac_of_spec": round(HBM_PROBE_GBS / 2 / HBM_PEAK_GBS, 4)}
    if t1 and t3:
        step_s = batch_bytes / alg_bps
        out.update({"read_bytes_per_step": int(t1 + t3), "read_gbs": round((t1 + t3) / step_s / 1e9, 2),
                    "frac": round((t1 + t3) / step_s / 1e9 / HBM_PEAK_GBS, 4),
                    "frac_of_probe": round((t1 + t3) / step_s / 1e9 / HBM_PROBE_GBS, 4),
                    "traffic_source": src})
    return out


# -------------------------------------------------------------- pipeline --
def lane_occupancy(arena_res, R, B, need, lanes, period=1):
    """Chains in flight per steady-state K3 launch, from the collected cut
    lists: batch x is in its t-th launch (t < need) in launch x + t, and a
    chunk of `nfull` full message blocks is still in the order list then iff
    t == 0 or nfull > t * B (K2c drops it after the launch that finishes it).
    Launch m holds batches m, m-1, .., m-need+1 (arena (m - t) % R).  With a
    K3 period P, B is the launch's budget and P batches join each launch:
    launch m holds the P arenas (mP - tP - q) % R, q < P, in their t-th."""
    per_arena = []
    for i in range(R):
        res = arena_res.get(i)
        if res is None:
            return None
        nf = np.concatenate([((np.diff(np.concatenate([[0], r.cut_ends.astype(np.int64)])) + 8) >> 6)
                             for r in res if r.n_chunks] or [np.zeros(0, np.int64)])
        per_arena.append([int(nf.size) if t == 0 else int(np.count_nonzero(nf > t * B))
                          for t in range(need)])
    active = [sum(per_arena[(m * period - t * period - q) % R][t] for t in range(need) for q in range(period))
              for m in range(R)]
    return {"active_chains_mean": round(float(np.mean(active)), 1), "active_chains_max": int(max(active)),
            "lanes": lanes, "occupancy_mean": round(float(np.mean(active)) / lanes, 4),
            "occupancy_max": round(max(active) / lanes, 4)}


def cpu_throttle():
    """(nr_throttled, throttled_usec) of this process's cgroup, or None: a
    CPU quota that runs out stalls the host mid-window."""
    for path, us in (("/sys/fs/cgroup/cpu.stat", "throttled_usec"), ("/sys/fs/cgroup/cpu/cpu.stat", None),
                     ("/sys/fs/cgroup/cpu,cpuacct/cpu.stat", None)):
        try:
            st = dict(line.split() for line in open(path))
        except (OSError, ValueError):
            continue
        t = int(st[us]) if us else int(st.get("throttled_time", 0)) // 1000
        return int(st.get("nr_throttled", 0)), t
    return None


def steady(eng, arenas, offs, lens, R, steps, warmup, dist, dev, before_submit=None, aliased=False):
    """Fill to R in flight, W warm-up steps, K timed steps (submit one into
    the next arena of the ring, then collect the oldest batch), then the
    drain.  A batch reuses the arena of the batch R before it while that one
    is still in the pipeline: hbx_input_after_oldest orders its scan (and an
    --e2e copy) after the launch that finishes the older batch, on the GPU,
    so the host collecting later never holds an arena back.  Returns
    timings, the window's launch counts and results."""
    order = deque()  # arena index of every pending batch, oldest first
    state = {"j": 0, "t_sub": 0.0, "t_col": 0.0, "subs": [], "cols": [], "parts": []}
    arena_res = {}

    def submit():
        t = time.perf_counter()
        i = state["j"] % R
        if len(order) >= R and not aliased:  # arena i still holds the oldest pending batch
            eng.input_after_oldest()
        t_a = time.perf_counter()
        if before_submit:
            before_submit(i)
        eng.submit_device(arenas[i].data_ptr(), offs, lens)
        state["parts"].append((t_a - t, getattr(eng, "alloc_s", 0.0), time.perf_counter() - t_a))
        order.append(i)
        state["j"] += 1
        dt = time.perf_counter() - t
        state["t_sub"] += dt
        state["subs"].append(dt)

    def collect():
        t = time.perf_counter()
        i = order.popleft()
        res = eng.wait()
        arena_res[i] = res
        dt = time.perf_counter() - t
        state["t_col"] += dt
        state["cols"].append(dt)
        return i, res

    torch.cuda.synchronize(dev)
    t_fill = time.perf_counter()
    for _ in range(R):
        submit()
    for _ in range(warmup):
        submit()
        collect()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.stage_totals(reset=True)  # everything before the window is complete and harvested
    eng.host_call_max(reset=True)
    state["t_sub"] = state["t_col"] = 0.0
    eng.wait_s = 0.0
    thr0 = cpu_throttle()
    t0 = time.perf_counter()
    last = None
    window = []
    for _ in range(steps):
        submit()
        last = collect()
        window.append(last)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    subs = np.array(state["subs"][-steps:]) * 1e3
    cols = np.array(state["cols"][-steps:]) * 1e3
    host = {"submit_ms": state["t_sub"] / steps * 1e3, "collect_ms": state["t_col"] / steps * 1e3,
            "in_hbx_wait_ms": eng.wait_s / steps * 1e3,
            "submit_ms_median_max": [round(float(np.median(subs)), 4), round(float(subs.max()), 4)],
            "submit_slowest_step": int(subs.argmax()),
            "slowest_submit_fence_alloc_call_ms": [round(x * 1e3, 4) for x in state["parts"][len(state["parts"]) - steps + int(subs.argmax())]],
            "collect_ms_max": round(float(cols.max()), 4),
            "collect_slowest_step": int(cols.argmax())}
    hc = eng.host_call_max()
    host["library_slowest_call_ms"] = {"h2d_copy": round(float(hc[0]), 4), "submit": round(float(hc[1]), 4)}
    thr1 = cpu_throttle()
    if thr0 and thr1:
        host["cpu_throttled_n_ms"] = [thr1[0] - thr0[0], round((thr1[1] - thr0[1]) / 1e3, 3)]
    if dist:
        dist.barrier()
    tot_ms, tot_n = eng.stage_totals()
    probe_raw = eng.k3_wave_times() if eng.knobs().get("k3_probe") else None  # the window's last launch
    probe = k3_probe_stats(probe_raw) if probe_raw is not None else None
    t_d = time.perf_counter()
    drained = None
    while order:
        drained = collect()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    return {"el": t1 - t0, "drain": t2 - t_d, "fill_to_drained": t2 - t_fill,
            "batches_total": state["j"], "tot_ms": tot_ms, "tot_n": tot_n,
            "last": last, "window": window, "drained": drained, "arena_res": arena_res, "host": host, "probe": probe,
            "probe_raw": probe_raw}


def k3_probe_stats(w):
    """Summary of one K3 launch's per-wave records (engine.k3_wave_times), µs."""
    w = w.astype(np.int64)
    busy = w[(w[:, 1] & ((1 << 56) - 1)) != 0]  # waves that ran a group (start-up stamped)
    if not len(busy):
        return None
    t0 = int(w[w[:, 0] != 0][:, 0].min())
    us = lambda x: np.round(np.asarray(x, np.float64) * 0.01, 1)  # noqa: E731  100 MHz ticks
    low56 = (1 << 56) - 1
    start = us(busy[:, 0] - t0)
    setup = us((busy[:, 1] & low56) - busy[:, 0])
    end = us(busy[:, 2] - t0)
    R = busy[:, 3] & 0xffff
    xcc = busy[:, 1] >> 56
    hw = busy[:, 3] >> 32
    simd, cu, se = (hw >> 4) & 3, (hw >> 8) & 0xf, (hw >> 13) & 3
    q = lambda a: [float(np.min(a)), float(np.median(a)), float(np.max(a))]  # noqa: E731
    full = R == R.max()
    out = {"busy_waves": int(len(busy)), "span_us": float(us(int(w[:, 2].max()) - t0)),
           "start_us_min_med_max": q(start), "startup_us_min_med_max": q(setup), "end_us_min_med_max": q(end),
           "R_min_med_max": q(R), "full_slice_waves": int(full.sum()),
           "full_slice_end_us_min_med_max": q(end[full]) if full.any() else None}
    for name, key in (("xcc", xcc), ("se", se), ("simd", simd)):
        out[f"full_end_us_by_{name}"] = {int(k): q(end[full & (key == k)]) for k in np.unique(key[full])}
    # slowest full-slice waves: where they ran
    order = np.argsort(-end)
    out["slowest10"] = [{"end_us": float(end[i]), "xcc": int(xcc[i]), "se": int(se[i]), "cu": int(cu[i]),
                         "simd": int(simd[i]), "R": int(R[i])} for i in order[:10]]
    return out


K3_VALU_FLOOR_CYCLES = 320 * SIMD_CYCLES_PER_VALU  # one MD5 block's 320 VALU at one wave per SIMD
# K1's whole mix (SDWA add/sub, v_lshl_add, v_max3, v_dot4, DPP adds) issues
# at 4.19-4.20 cycles per wave-instruction per SIMD at four waves per SIMD
# (profiles/r03b/valu_issue.txt): K1's per-SIMD issue ceiling
K1_CYCLES_PER_VALU_4W = 4.20


def lifetime_leg(eng, arenas, offs, lens, R, B, lead, nfull, head, dist, gpu, period=1):
    """Where a batch's lifetime goes (verdict r04 item 3), from a short
    probed run after the timed window (hbx_set_k3_probe: per-wave s_memtime /
    s_memrealtime stamps around the first group's cooperative phase; the
    probe changes no result).  Throughput = R resident batches / lifetime, and
    lifetime / the serial floor of the longest chunk = staging x launch
    overhead x lead:
      staging         cycles per block / the 1,312 of 320 VALU at 4.1 cycles
      launch_overhead K3's average launch / (B x cycles per block / clock)
      lead            R / (R - lead): batches resident but not in K3
    plus the step's excess over K3's launch (the scan loop).  With a K3
    period P, B is the launch's budget (P x the slice), a launch spans P
    steps, and a batch waits up to P - 1 more submits to join."""
    eng.set_k3_probe(True)
    try:  # the records of the last launch of the steps, a steady-state one (not the drain's)
        w = steady(eng, arenas, offs, lens, R, max(3, period), max(3, period), dist, gpu)["probe_raw"].astype(np.int64)
    finally:
        eng.set_k3_probe(False)
    blocks = w[:, 7] & 0xffffffff
    polls = w[:, 7] >> 32  # the wave's polls that found its producer's stage not yet written
    keep = blocks > 0
    coop, blocks, polls = w[keep], blocks[keep], polls[keep]
    if not len(coop):
        return None
    R_w = coop[:, 3] & 0xffff
    sel = R_w == R_w.max()
    full, fblocks, fpolls = coop[sel], blocks[sel], polls[sel]
    cyc = (full[:, 5] - full[:, 4]).astype(np.float64)
    ticks = (full[:, 6] - (full[:, 1] & ((1 << 56) - 1))).astype(np.float64)
    cpb = float(np.median(cyc / fblocks))
    # the slowest tenth of the full-slice waves (by cycles per block) against the
    # rest: do they wait for their producer (polls), or issue slower?
    per = cyc / fblocks
    slow = per >= np.quantile(per, 0.9)
    stage_wait = {"polls_per_wave_min_med_max": [int(fpolls.min()), float(np.median(fpolls)), int(fpolls.max())],
                  "polls_per_1000_blocks_median": round(float(np.median(fpolls / fblocks * 1000)), 3),
                  "slowest_tenth_cycles_per_block_median": round(float(np.median(per[slow])), 1),
                  "slowest_tenth_polls_median": float(np.median(fpolls[slow])),
                  "rest_polls_median": float(np.median(fpolls[~slow])) if (~slow).any() else None,
                  "poll_sleep_cycles": 64}
    ghz = float(np.median(cyc / np.maximum(ticks, 1) * 0.1))
    launch_ms = float(head["roofline"]["avg_launch_ms"])
    hashing_ms = B * cpb / ghz * 1e-6
    step_ms = float(head["ms_per_step"])
    floor_ms = nfull * K3_VALU_FLOOR_CYCLES / ghz * 1e-6
    busy = int((w[:, 1] & ((1 << 56) - 1) != 0).sum())
    return {
        "source": "bench.py lifetime_leg: hbx_set_k3_probe, the last launch of 3 steady-state steps after the timed "
                  "window (full-slice waves, first group's cooperative phase)",
        "cycles_per_block": round(cpb, 1), "clock_ghz": round(ghz, 4),
        "floor_cycles_per_block": K3_VALU_FLOOR_CYCLES, "full_slice_waves": int(len(full)),
        "staging": round(cpb / K3_VALU_FLOOR_CYCLES, 4),
        "launch_overhead": round(launch_ms / hashing_ms, 4),
        "lead": round(R / max(1, R - lead - period + 1), 4),
        "step_over_launch": round(step_ms * period / launch_ms, 4),
        "lifetime_ms": round(R * step_ms, 2), "serial_floor_ms": round(floor_ms, 2),
        "lifetime_over_floor": round(R * step_ms / floor_ms, 4),
        "k3_busy_waves": busy,
        "stage_wait": stage_wait,
    }


def max_over_ranks(x, dist, dev, op="max"):
    if not dist:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.MIN)
    return float(t.item())


def run_workload(a, name, eng, arenas, offs, lens, R, B, need, lanes, dist, gpu, dev, world, rank,
                 job_batch_bytes, check_threads, before_submit=None, period=1):
    """One steady-state measurement; returns the JSON fields of its line.
    `gpu` is this rank's device, `dev` the device of the reductions."""
    r = steady(eng, arenas, offs, lens, R, a.steps, a.warmup, dist, gpu, before_submit,
               aliased=a.alias_depth > 0)
    el = max_over_ranks(r["el"], dist, dev)
    tot_ms, tot_n = r["tot_ms"], r["tot_n"]
    k1_n, k3_n = int(tot_n[0]), int(tot_n[3])
    # one K3 launch per `period` submits (a.steps is a multiple of the period)
    window_exact = k1_n == a.steps and k3_n * period == a.steps
    if not window_exact:
        raise RuntimeError(f"{name}: timed window holds {k1_n} K1 and {k3_n} K3 launches, expected "
                           f"{a.steps} and {a.steps // period} (a forced drain or an empty batch inside the window)")
    rank_batch = int(sum(int(n) for n in lens))
    avg_ms = tot_ms / np.maximum(tot_n, 1)
    # dominant kernel: K3.  Algorithmic bytes per launch = the rank's batch
    # bytes x the K3 period (one K3 launch per `period` steps advances every
    # chain in flight; in steady state the chains hashed per launch add up to
    # `period` batches), over the K3 launches of the window only.
    per_launch = a.steps * rank_batch / k3_n
    achieved = per_launch / (avg_ms[3] * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic(KERNEL_OF["k3_block_md5"], per_launch, rank_batch)
    k1_gbs = (a.steps * rank_batch / k1_n) / (avg_ms[0] * 1e-3) / 1e9 if tot_ms[0] > 0 else 0.0
    k3_bps = a.steps * rank_batch / (tot_ms[3] * 1e-3) if tot_ms[3] > 0 else 0.0
    res = r["last"][1]
    n_chunks = sum(x.n_chunks for x in res)
    longest = max((int(np.max(np.diff(np.concatenate([[0], x.cut_ends]).astype(np.int64))))
                   for x in res if x.n_chunks), default=0)
    check = None
    n_checked = 0
    if not a.no_check:  # outside the timer: the last K batches collected in the window (each
        # its own arena while K <= R: the arenas are read-only inputs), and the last one
        # drained (completed by the forced drain launch); every file of each
        ok = True
        for i, got in r["window"][-max(1, min(a.check_batches, R)):]:
            ok = ok and oracle_check(arenas[i], offs, lens, got, check_threads)
            n_checked += 1
        if r["drained"] is not None:
            ok = ok and oracle_check(arenas[r["drained"][0]], offs, lens, r["drained"][1], check_threads)
            n_checked += 1
        check = bool(max_over_ranks(1.0 if ok else 0.0, dist, dev, op="min") == 1.0)
    value = a.steps * job_batch_bytes / el / GIB
    drain = max_over_ranks(r["drain"], dist, dev)
    fill = max_over_ranks(r["fill_to_drained"], dist, dev)
    out = {
        "value": round(value, 3), "ms_per_step": round(el / a.steps * 1e3, 4),
        "drain_ms": round(drain * 1e3, 2),
        "fill_drain_gibs": round(r["batches_total"] * job_batch_bytes / fill / GIB, 3),
        "chunks_per_gpu_step": n_chunks,
        "longest_chunk_bytes": longest,
        # the contract's HBM roofline of the dominant kernel; what actually
        # limits K3 ("limiter"): its instruction stream at one
        # wave per SIMD and, meeting it, its loads from 32k chains scattered
        # over the arenas, pushed out by K1's HBM traffic
        "roofline": {"kernel": "k3_block_md5", "bound": "hbm", "achieved": round(achieved, 2),
                     "limiter": "valu-issue of one MD5 wave per SIMD (5 dependent VALU per step) meeting the "
                                "loads of 32k chains scattered over the arenas (tools/ubench/hbm_streams: "
                                "2.65-2.80 ms per 8 GiB without the MD5), plus K1's HBM traffic beside it",
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic, "traffic_source": traffic_src, "launches": k3_n,
                     "avg_launch_ms": round(float(avg_ms[3]), 4),
                     "algorithmic_bytes_per_launch": int(per_launch), "window_only": True},
        "k1_roofline": {"achieved": round(k1_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(k1_gbs / HBM_PEAK_GBS, 4), "avg_launch_ms": round(float(avg_ms[0]), 4)},
        # the whole path's issue bound: K1 + K3 VALU wave-instructions per
        # step over the chip's measured issue ceiling for their classes at the
        # spec clock (the box runs power-capped at ~2.09 GHz while pipelined)
        "valu_roofline": {"bound": "valu-issue", "unit": "wave-instr/s per GPU",
                          "achieved": round(rank_batch * (K1_WAVE_VALU_PER_BYTE + K3_WAVE_VALU_PER_BYTE)
                                            / (el / a.steps), 0),
                          "peak": round(VALU_PEAK_WAVE_INSTR, 0),
                          "frac": round(rank_batch * (K1_WAVE_VALU_PER_BYTE + K3_WAVE_VALU_PER_BYTE)
                                        / (el / a.steps) / VALU_PEAK_WAVE_INSTR, 4),
                          "k1_valu_per_byte": round(K1_WAVE_VALU_PER_BYTE * 64, 3),
                          "k3_valu_per_byte": round(K3_WAVE_VALU_PER_BYTE * 64, 3),
                          "simd_cycles_per_valu": SIMD_CYCLES_PER_VALU,
                          "source": VALU_SOURCE},
        # bytes the step actually reads (K1 + K3, PMC FETCH_SIZE) against the
        # spec peak, and the algorithmic rate against the two-read ceiling
        "path_roofline": path_roofline(a.steps * rank_batch / el, rank_batch),
        "k3_lanes": lane_occupancy(r["arena_res"], R, B * period, need, lanes, period),
        "kernel_ms_per_step": {n: round(float(v) / a.steps, 4) for n, v in zip(KNAMES, tot_ms)},
        "window_launches": {n: int(v) for n, v in zip(KNAMES, tot_n)},
        # host time per step inside the window (rank 0's): submit, and collect (incl. any wait)
        "host_ms_per_step": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r["host"].items()},
    }
    if r["probe"] is not None:
        out["k3_probe"] = r["probe"]
    if check is not None:
        out["check_vs_oracle"] = check
        out["checked_batches_per_gpu"] = n_checked
    return out


ARENA_SLACK = 64 << 20  # per resident batch beyond its packed bytes (allocator rounding)


def residency_plan(files, file_mib, world, rank, scaling="strong", free_bytes=0, hbm_frac=0.95,
                   ranks_per_device=1, arenas=0, md5_slice=-1, join_lag=0, lead=-1, e2e=False,
                   alias_depth=0, k3_period=0, steps=0):
    """The pipeline each rank runs.  Files of the job:
    `files` x `file_mib` MiB; strong scaling gives this rank its LPT share of
    each step's files (independent files, store.go:84-199), weak a whole
    batch.  The schedule itself (R resident batches, slice B, join lag, lead,
    K3 period, launches per batch `need`) comes from the library's planner,
    hbx_plan_pipeline (include/hbxgpu.h), so a cgo caller gets exactly the
    plan this bench runs; tests/test_plan.py checks it against the round-5
    Python planner at N = 1..8.  Pure host arithmetic (no GPU) for a given
    free_bytes."""
    from hashbox_amd import plan_pipeline
    from hashbox_amd.shard import lpt_assign
    import workloads as W
    fbytes = file_mib << 20
    job_lens = [fbytes] * files
    mine = lpt_assign(job_lens, world)[rank] if scaling == "strong" else list(range(files))
    lens = [job_lens[i] for i in mine]
    if not lens:
        raise ValueError(f"rank {rank} has no files: --files {files} < world {world}")
    nf = len(lens)
    offs, total = W.pack_layout(lens)
    req = dict(n_files=nf, arena_bytes=total, longest_file=max(lens), free_bytes=free_bytes, hbm_frac=hbm_frac,
               ranks_per_device=ranks_per_device, steps=steps, arenas=arenas, md5_slice=md5_slice,
               join_lag=join_lag, lead=lead, k3_period=k3_period, host_input=e2e)
    if alias_depth > 0:  # diagnostics: D in flight over the physical arenas
        p = plan_pipeline(**dict(req, arenas=alias_depth))
        try:
            physical = plan_pipeline(**req)["resident"]
        except ValueError:  # too few physical arenas for a plan of their own
            physical = arenas
    else:
        p = plan_pipeline(**req)
        physical = p["resident"]
    return {"lib_plan": p, "mine": mine, "lens": lens, "files_per_gpu": nf, "join_lag": p["join_lag"], "lead": p["lead"],
            "offs": offs, "arena_bytes": total, "R": p["resident"], "physical_arenas": physical,
            "B": p["md5_slice"], "need": p["launches_per_batch"], "k3_period": p["k3_period"],
            "hbm_bytes": physical * (total + ARENA_SLACK), "file_bytes": fbytes}


def check_host_bytes(plan, world_on_host=1):
    """Host memory the oracle check legs take on one rank (a copy of one batch
    plus the oracle's outputs), times the ranks sharing the host."""
    return world_on_host * (int(plan["arena_bytes"]) + 64 * int(plan["files_per_gpu"]) * 1024)


def main():
    a = parse()
    if a.k3_period > 0 and a.steps % a.k3_period:  # advisor r05: the window must hold whole K3 periods
        sys.exit(f"--k3-period {a.k3_period} must divide --steps {a.steps} (one K3 launch per period; the "
                 "timed window's launch count is asserted)")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != a.gpus and rank == 0:
        print(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    ndev = torch.cuda.device_count()  # counts only; does not initialise the GPU
    dev_idx = local % max(ndev, 1)
    dev = torch.device("cuda", dev_idx)
    dist = None
    if world > 1 or a.dist_always:
        import datetime
        import torch.distributed as dist
        to = datetime.timedelta(seconds=a.dist_timeout)
        if a.dist_backend == "nccl" and not a.plan_only:
            torch.cuda.set_device(dev_idx)
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        else:
            dist.init_process_group(a.dist_backend, timeout=to)
    red_dev = dev if (dist and a.dist_backend == "nccl" and not a.plan_only) else torch.device("cpu")

    # Per-rank setup.  Any failure here (a bad plan, out of memory, a HIP
    # error) is reported to every rank before the first barrier, so all exit
    # non-zero instead of leaving the others waiting until the timeout.
    err = None
    try:
        S = setup(a, rank, world, local_world, ndev, dev_idx, dev)
    except Exception as e:  # noqa: BLE001  reported below, then every rank exits
        import traceback
        traceback.print_exc()
        err = f"{type(e).__name__}: {e}"
        S = None
    ok = max_over_ranks(0.0 if err else 1.0, dist, red_dev, op="min") == 1.0
    if not ok:
        print(f"rank {rank}: setup failed ({err or 'on another rank'}); exiting", file=sys.stderr, flush=True)
        if dist:
            dist.destroy_process_group()
        sys.exit(1)
    if a.plan_only:
        P = S["plan"]
        mine = {"rank": rank, **{k: P[k] for k in ("files_per_gpu", "join_lag", "lead", "R", "physical_arenas",
                                                   "B", "need", "k3_period", "hbm_bytes", "file_bytes",
                                                   "arena_bytes")},
                "mine": P["mine"], "check_host_bytes": check_host_bytes(P)}
        plans = [mine]
        if dist:
            plans = [None] * world
            dist.all_gather_object(plans, mine)
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"plan_only": True, "world": world, "scaling": a.scaling, "plans": plans}), flush=True)
        return
    run(a, S, rank, world, local_world, dist, dev, red_dev)


def corpus_file_ids(a, P, rank):
    """Job file ids of this rank's files (workloads.fill_batch)."""
    return [int(j) for j in P["mine"]] if a.scaling == "strong" else [int(j) + a.files * rank for j in P["mine"]]


def setup(a, rank, world, local_world, ndev, dev_idx, dev):
    """Everything a rank prepares before the first barrier: its plan, arenas
    and engine (with every pipeline buffer reserved)."""
    if a.fail_rank == rank:
        raise RuntimeError(f"--fail-rank {rank}: injected setup failure")
    # ranks sharing one device (tests) share its HBM
    share = max(1, -(-local_world // max(ndev, 1)))
    if a.plan_only and a.free_gib > 0:  # planning for one device per rank
        free, share = int(a.free_gib * GIB), 1
    else:
        torch.cuda.set_device(dev_idx)
        free, _ = torch.cuda.mem_get_info(dev)
    P = residency_plan(a.files, a.file_mib, world, rank, a.scaling, free, a.hbm_frac, share, a.arenas,
                       a.md5_slice, a.join_lag, a.lead, a.e2e, a.alias_depth, a.k3_period, a.steps)
    if a.plan_only:
        return {"plan": P}
    from hashbox_amd import Engine
    import workloads as W
    lens, offs, total = P["lens"], P["offs"], P["arena_bytes"]
    R, B, need, lag = P["R"], P["B"], P["need"], P["join_lag"]
    cores = cpu_info()
    threads = a.cpu_threads or cores["usable"]
    if world > 1:  # ranks share the host's cores for the oracle check
        threads = max(1, threads // local_world)
    # one job corpus: file j of resident batch b has bytes from seed (seed, b,
    # j) on whichever rank holds it, so strong scaling splits the same files a
    # one-GPU run hashes (workloads.fill_batch); weak scaling gives every rank
    # job files of its own (j + files x rank)
    file_ids = corpus_file_ids(a, P, rank)
    arenas = W.corpus_arenas(P["physical_arenas"], total, offs, lens, file_ids, a.seed, dev, single=a.single_alloc)
    if a.alias_depth > 0:  # diagnostics: D in flight over the physical arenas
        arenas = [arenas[i % P["physical_arenas"]] for i in range(R)]
    ballast = torch.zeros(int(a.ballast_gib * GIB), dtype=torch.uint8, device=dev) if a.ballast_gib else None
    torch.cuda.synchronize(dev)
    eng = Engine(dev_idx)
    if a.k3_probe:  # the probe alone (hbx_set_k3_probe), no other HBX_* switch
        eng.set_k3_probe(True)
    # the library's plan (hbx_apply_plan): slice, join lag, K3 period, and every
    # batch slot, chain table and summary buffer of the pipeline allocated now
    # (an allocation inside the timed region would drain the streams)
    eng.apply_plan(P["lib_plan"], len(lens), sum(lens))
    k = eng.knobs()
    assert (k["md5_slice"], k["join_lag"], k["k3_period"]) == (B, lag, P["k3_period"]), k
    for _ in range(2):  # single-batch latency (one batch alone, synchronous call), untimed
        eng.chunk_hash_device(arenas[0].data_ptr(), offs, lens)
    latency = eng.stage_times()
    return {"plan": P, "arenas": arenas, "ballast": ballast, "eng": eng, "latency": latency, "cores": cores,
            "threads": threads}


def e2e_leg(a, eng, arenas, offs, lens, P, lanes, dist, dev, red_dev, world, rank, job_batch, threads):
    """The PCIe-inclusive rate (north_star: "the end-to-end rate including
    pinned hipMemcpyAsync H2D/D2H overlapped on a side stream must also be
    measured"): the same pipeline, but every step's batch starts in pinned
    host memory (hbx_alloc_pinned) and is copied into its arena by
    hbx_memcpy_h2d_async on the engine's scan stream, overlapped with the
    kernels of the batches before it; the cut lists, block IDs and content ids
    come back by the result stream's D2H copy (hbx_wait).  H2D-bound, so a
    shallow pipeline: R = lead + 2 resident arenas, two K3 launches per batch.
    Runs after the device-resident lines; the random batch is regenerated."""
    import copy
    import ctypes
    used = int(offs[-1]) + int(lens[-1])
    ld, lag = P["lead"], P["join_lag"]
    R_e = min(ld + 2, len(arenas))
    nfull = (min(P["file_bytes"], 8 << 20) + 8) >> 6
    B_e = -(-nfull // max(1, R_e - ld))
    need_e = -(-nfull // B_e)
    if need_e + lag > R_e:
        return None
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed + 7919 * rank)
    arenas[0].random_(0, 256, generator=g)
    hp = ctypes.c_void_p()
    if eng._L.hbx_alloc_pinned(used, ctypes.byref(hp)) != 0:
        raise RuntimeError("hbx_alloc_pinned failed")
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * used).from_address(hp.value))
        torch.from_numpy(host).copy_(arenas[0][:used])
        torch.cuda.synchronize(dev)
        eng.set_md5_slice(B_e)
        eng.set_k3_period(1)  # PCIe-bound, shallow: one launch per step

        def before(i):
            eng.memcpy_h2d_async(arenas[i].data_ptr(), hp.value, used)

        ae = copy.copy(a)
        ae.steps, ae.warmup = a.e2e_steps, min(a.warmup, 3)
        r = run_workload(ae, "e2e", eng, arenas[:R_e], offs, lens, R_e, B_e, need_e, lanes, dist, dev, red_dev,
                         world, rank, job_batch, threads, before)
    finally:
        eng._L.hbx_free_pinned(hp)
    keep = ("value", "ms_per_step", "drain_ms", "fill_drain_gibs", "kernel_ms_per_step", "window_launches",
            "host_ms_per_step", "check_vs_oracle")
    out = {k: r[k] for k in keep if k in r}
    out.update({"unit": "GiB/s", "steps": ae.steps, "warmup": ae.warmup,
                "what": "pinned host memory (hbx_alloc_pinned) -> hbx_memcpy_h2d_async on the scan stream -> "
                        "K1/K2/K3/K4 -> D2H of cut lists + block IDs + content ids into host memory; "
                        "every step copies its whole batch over PCIe",
                "h2d_bytes_per_step_per_gpu": used, "pipeline_depth": R_e, "md5_slice_blocks": B_e,
                "launches_per_batch": need_e})
    return out


def run(a, S, rank, world, local_world, dist, dev, red_dev):
    """The measurement proper: steady-state windows, checks, the JSON line."""
    from hashbox_amd import _lib
    import workloads as W
    P, eng, arenas, latency = S["plan"], S["eng"], S["arenas"], S["latency"]
    lens, offs, total = P["lens"], P["offs"], P["arena_bytes"]
    R, B, need, lag, lead, nf = P["R"], P["B"], P["need"], P["join_lag"], P["lead"], P["files_per_gpu"]
    per = P["k3_period"]
    n_phys = P["physical_arenas"]
    fbytes = P["file_bytes"]
    cores, threads = S["cores"], S["threads"]
    job_batch = a.files * fbytes if a.scaling == "strong" else a.files * fbytes * world
    lanes = torch.cuda.get_device_properties(dev).multi_processor_count * 4 * 64

    before = None
    host_pin = None
    if a.e2e:  # the batch starts in pinned host memory; each step copies it into its arena
        import ctypes
        used = int(offs[-1]) + lens[-1]
        hp = ctypes.c_void_p()
        if eng._L.hbx_alloc_pinned(used, ctypes.byref(hp)) != 0:
            raise RuntimeError("hbx_alloc_pinned failed")
        host_pin = hp
        np.ctypeslib.as_array((ctypes.c_uint8 * used).from_address(hp.value))[:] = \
            arenas[0][:used].cpu().numpy()

        def before(i):
            eng.memcpy_h2d_async(arenas[i].data_ptr(), host_pin.value, used)

    lines = {}
    workloads = ["random", "zipf"] if a.workload == "both" else [a.workload]
    if a.e2e:  # each step copies the random batch in: one line
        workloads = ["random"]
    zipf_repeat = None
    for wl in workloads:
        if wl == "zipf":
            zipf_repeat = W.zipf_fill(arenas, int(offs[-1]) + lens[-1], a.seed + 4 + 7919 * rank)
        lines[wl] = run_workload(a, wl, eng, arenas, offs, lens, R, B, need, lanes, dist, dev, red_dev,
                                 world, rank, job_batch, threads, before, per)
        if zipf_repeat is not None and wl == "zipf":
            lines[wl]["repeat_fraction"] = round(zipf_repeat, 4)

    life = None
    if not a.no_lifetime and a.alias_depth == 0 and not a.e2e:
        nfull = (min(fbytes, 8 << 20) + 8) >> 6
        life = lifetime_leg(eng, arenas, offs, lens, R, B * per, lead, nfull, lines[workloads[0]], dist, dev, per)
        if zipf_repeat is not None:  # the arenas hold the Zipf corpus now: the probe ran over it
            life["probed_over"] = "the Zipf arenas (MD5 cycles per block do not depend on the bytes)"

    e2e = None
    if a.e2e_steps > 0 and not a.e2e and a.alias_depth == 0:
        e2e = e2e_leg(a, eng, arenas, offs, lens, P, lanes, dist, dev, red_dev, world, rank, job_batch, threads)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.e2e:
        # rebuild the random batch 0 (the arenas may hold the Zipf corpus now)
        W.fill_batch(arenas[0], 0, offs, lens, corpus_file_ids(a, P, rank), a.seed)
        k = min(a.cpu_files, nf)
        host = arenas[0][:int(offs[k - 1]) + lens[k - 1]].cpu().numpy()
        cpu = cpu_baseline([host[int(offs[i]):int(offs[i]) + lens[i]] for i in range(k)], threads, cores)
        del host

    head = lines[workloads[0]]
    if a.e2e:
        metric = ("end-to-end GiB/s, pinned host memory -> HBM (H2D on the scan stream) -> chunk lists + "
                  "block IDs in host memory, pipelined MD5")
    else:
        metric = METRIC
    out = {
        "metric": metric,
        "value": head["value"],
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic: uniform random bytes generated on the device (torch Generator), {R} distinct "
                f"resident batches per GPU, resident in HBM before timing",
        "config": {"workload": f"{a.files} x {a.file_mib} MiB random buffers per step, rollsum split + MD5 "
                               "block IDs + file content ids, device-resident (configs[1]"
                               + ((", sharded by file across GPUs: configs[2])" if a.scaling == "strong"
                                   else " on every GPU, each rank its own files)") if world > 1 else ")"),
                   "files_per_step": a.files, "files_per_gpu": nf, "file_bytes": fbytes,
                   "md5_slice_blocks": B, "pipeline_depth": R, "launches_per_batch": need,
                   "scan_lead": lead, "join_lag": lag, "k3_period": per,
                   "parallelism": f"file-sharded x{world} ({a.scaling} scaling; independent HIP streams, "
                                  "no data-path collective)",
                   "seeds": f"one job corpus generated on the devices: file j of resident batch b from seed "
                            f"({a.seed}, b, j) on whichever rank holds it"
                            + (", so the ranks split the files a one-GPU run hashes" if a.scaling == "strong"
                               else ", j + files x rank under weak scaling")
                            + f"; Zipf corpus seed {a.seed + 4} + 7919 x rank"},
    }
    out.update({k: v for k, v in head.items() if k not in ("value", "ms_per_step")})
    out["single_batch"] = {"ms": round(float(latency[4]), 3),
                           "gibs": round(sum(lens) / GIB / (float(latency[4]) * 1e-3), 3),
                           "stages_ms": [round(float(x), 3) for x in latency]}
    out["cpu_baseline"] = cpu
    if life is not None:
        out["lifetime"] = life
        # the two loops' VALU ceilings, each for its own issue mode
        # (profiles/r03b/valu_issue.txt): K3 is bound by ONE wave's issue
        # (a chain's speed at fixed residency), K1 by the SIMD's issue at
        # four waves of an all-half-rate mix, on the CUs K3 leaves
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        k3_cus = -(-life["k3_busy_waves"] // 4)
        k1_simds = max(1, cus - k3_cus) * 4
        k1_ms = float(head["kernel_ms_per_step"]["k1_digest_scan"])
        k1_need = sum(int(n) for n in lens) * K1_WAVE_VALU_PER_BYTE * K1_CYCLES_PER_VALU_4W
        out["valu_roofline"]["k3"] = {
            "bound": "one wave's VALU issue (one MD5 wave per SIMD; a chain's speed)",
            "peak_cycles_per_block": K3_VALU_FLOOR_CYCLES, "achieved_cycles_per_block": life["cycles_per_block"],
            "frac": round(K3_VALU_FLOOR_CYCLES / life["cycles_per_block"], 4)}
        out["valu_roofline"]["k1"] = {
            "bound": f"SIMD issue at four waves per SIMD, half-rate mix ({K1_CYCLES_PER_VALU_4W} cycles per "
                     "wave-VALU), on the CUs K3 leaves",
            "simds": k1_simds, "launch_ms": k1_ms, "clock_ghz": life["clock_ghz"],
            "frac": round(k1_need / (k1_simds * k1_ms * 1e-3 * life["clock_ghz"] * 1e9), 4)}
    if e2e is not None:
        out["e2e"] = e2e
    if "zipf" in lines and workloads[0] != "zipf":
        out["zipf"] = dict(lines["zipf"], workload=f"{a.files} x {a.file_mib} MiB Zipf-duplicated buffers "
                                                   "(configs[3] scheme), device-resident")
    if a.alias_depth > 0:
        out["aliased"] = {"depth": R, "physical_arenas": n_phys,
                          "note": "diagnostic: in-flight batches share arenas; not a headline"}
    out["lib"] = dict(_lib.identity(), knobs=eng.knobs())
    if rank == 0:
        print(json.dumps(out), flush=True)
    if host_pin is not None:
        eng._L.hbx_free_pinned(host_pin)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

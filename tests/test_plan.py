"""The pipeline planner in the C-ABI (hbx_plan_pipeline, include/hbxgpu.h)
against the round-5 Python planner it replaced in bench.py (verdict r05 item
3: the operating point the bench line quotes must be what a cgo caller of
the library gets).  Pure host arithmetic: runs without a GPU.

`_py_plan` below is bench.residency_plan's schedule as of round 5 (commit
526942d, bench.py:587-654), kept as the reference, with round 6's one change:
the default lead is the join lag at 64 or more files per GPU."""
import pytest

ARENA_SLACK = 64 << 20
GIB = 1 << 30


def _py_plan(nf, total, fbytes, free_bytes, hbm_frac=0.95, ranks_per_device=1, arenas=0, md5_slice=-1,
             join_lag=0, lead=-1, e2e=False, k3_period=0, steps=0):
    lag = join_lag if join_lag > 0 else 2
    if k3_period > 0:
        per = k3_period
    else:
        per = next((p for p in (4, 2) if steps <= 0 or steps % p == 0), 1) if nf < 32 and not e2e else 1
    # round 6: lead = lag at 64+ files per GPU (device input), lag + 1 below
    ld = lead if lead >= 0 else lag + (0 if nf >= 64 and not e2e else 1)
    nfull = (min(fbytes, 8 << 20) + 8) >> 6
    r_fit = max(ld + 1, int(free_bytes * hbm_frac / max(1, ranks_per_device)) // (total + ARENA_SLACK))
    if e2e:
        r_fit = min(r_fit, ld + 2)

    def slice_for(R):
        launches = max(1, (R - ld - per + 1) // per)
        return -(-nfull // (launches * per))
    if md5_slice < 0:
        R = arenas if arenas > 0 else r_fit
        B = slice_for(R)
    else:
        B = md5_slice
        R = arenas if arenas > 0 else min((1 if B == 0 else -(-nfull // (B * per))) * per + ld + per - 1, r_fit)
    need = 1 if B == 0 else -(-nfull // (B * per))
    if need * per + lag + per - 1 > R:
        raise ValueError("depth")
    return {"resident": R, "md5_slice": B, "join_lag": lag, "lead": ld, "k3_period": per,
            "launches_per_batch": need, "hbm_bytes": R * (total + ARENA_SLACK)}


def _layout(nf, fbytes):
    import workloads as W
    return W.pack_layout([fbytes] * nf)[1]


@pytest.mark.parametrize("world", range(1, 9))
@pytest.mark.parametrize("files", [8, 16, 32, 64])
def test_c_plan_equals_python_plan(world, files):
    """bench's default at every world size and job size: strong scaling
    (files / world per rank, LPT), weak scaling (files per rank), several
    free-memory sizes and steps counts."""
    from hashbox_amd import plan_pipeline
    from hashbox_amd.shard import lpt_assign
    fbytes = 128 << 20
    shares = {len(p) for p in lpt_assign([fbytes] * files, world) if p} | {files}
    for nf in sorted(shares):
        total = _layout(nf, fbytes)
        for free_gib in (268.0, 282.5, 40.0):
            for steps in (0, 20, 200, 7, 6):
                want = _py_plan(nf, total, fbytes, int(free_gib * GIB), steps=steps)
                got = plan_pipeline(nf, total, fbytes, free_bytes=int(free_gib * GIB), steps=steps)
                assert got == want, (world, nf, free_gib, steps)


@pytest.mark.parametrize("kw", [
    {}, {"arenas": 40}, {"md5_slice": 4096}, {"md5_slice": 0}, {"join_lag": 1}, {"join_lag": 3, "lead": 5},
    {"lead": 2}, {"k3_period": 2}, {"k3_period": 8, "md5_slice": 64}, {"e2e": True}, {"hbm_frac": 0.78},
    {"ranks_per_device": 2}, {"arenas": 12, "md5_slice": 16384}, {"md5_slice": 9, "k3_period": 3},
])
@pytest.mark.parametrize("nf,fmib", [(64, 128), (8, 128), (4, 16), (100, 1), (1, 1024)])
def test_c_plan_overrides(kw, nf, fmib):
    """Every override bench.py exposes, on several batch shapes (including
    files below 8 MiB, whose chains are shorter)."""
    from hashbox_amd import plan_pipeline
    fbytes = fmib << 20
    total = _layout(nf, fbytes)
    free = int(268 * GIB)
    ckw = dict(kw)
    e2e = ckw.pop("e2e", False)
    try:
        want = _py_plan(nf, total, fbytes, free, e2e=e2e, **ckw)
    except ValueError:
        with pytest.raises(ValueError, match="pipeline depth"):
            plan_pipeline(nf, total, fbytes, free_bytes=free, host_input=e2e, **ckw)
        return
    assert plan_pipeline(nf, total, fbytes, free_bytes=free, host_input=e2e, **ckw) == want


def test_c_plan_refusals():
    from hashbox_amd import plan_pipeline
    with pytest.raises(ValueError):
        plan_pipeline(0, 1 << 20, 1 << 20, free_bytes=GIB)
    with pytest.raises(ValueError):
        plan_pipeline(8, 1 << 30, 128 << 20, free_bytes=GIB, join_lag=5)
    with pytest.raises(ValueError):
        plan_pipeline(8, 1 << 30, 128 << 20, free_bytes=GIB, k3_period=9)
    with pytest.raises(ValueError):  # no context to ask for the free memory
        plan_pipeline(8, 1 << 30, 128 << 20, free_bytes=0)
    with pytest.raises(ValueError):  # 3 arenas cannot hold 4 launches + lag 2
        plan_pipeline(8, 1 << 30, 128 << 20, free_bytes=GIB, arenas=3, md5_slice=32768, k3_period=1)


def test_bench_plan_is_the_library_plan():
    """bench.residency_plan hands the library's plan through unchanged."""
    import bench
    from hashbox_amd import plan_pipeline
    P = bench.residency_plan(64, 128, 8, 3, free_bytes=int(282 * GIB), steps=20)
    lp = plan_pipeline(P["files_per_gpu"], P["arena_bytes"], 128 << 20, free_bytes=int(282 * GIB), steps=20)
    assert P["lib_plan"] == lp
    assert (P["R"], P["B"], P["join_lag"], P["lead"], P["k3_period"], P["need"]) == (
        lp["resident"], lp["md5_slice"], lp["join_lag"], lp["lead"], lp["k3_period"], lp["launches_per_batch"])
    assert P["files_per_gpu"] == 8 and P["k3_period"] == 4 and P["join_lag"] == 2 and P["lead"] == 3

"""GPU, more than one process: the N>1 paths run as the driver launches them
(torch.distributed.run, one process per rank), here with gloo and every rank
on cuda:0 of the one-GPU box.

* bench.py at its default (strong scaling, configs[2]: each step's files
  LPT-split across the ranks) and --scaling weak, world 2, and strong at
  world 1, each with its pinned-host e2e leg: the window
  holds exactly K K1/K3 launches per rank and every rank's checked batches
  are bit-exact (check_vs_oracle, min over ranks).
* bench.py over RCCL (the nccl backend the driver uses) at world 1.
* hashbox_amd.multi.run_sharded driving the pipelined Engine on each rank:
  the gathered per-file results equal the oracle's for every file."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[-1])


BENCH = ["bench.py", "--files", "4", "--file-mib", "16", "--steps", "6", "--warmup", "2", "--arenas", "8",
         "--md5-slice", "32768", "--no-cpu-baseline", "--dist-backend", "gloo", "--cpu-threads", "4"]


@pytest.mark.parametrize("nproc,scaling", [(2, None), (2, "weak"), (1, "strong")])
def test_bench_through_torchrun(nproc, scaling):
    """scaling None = bench.py's default, which must be strong (configs[2]).
    Every line carries the pinned-host e2e leg, checked against the oracle."""
    d = _torchrun(nproc, BENCH + ["--gpus", str(nproc)] + (["--scaling", scaling] if scaling else []))
    scaling = scaling or "strong"
    assert d["n_gpus"] == nproc and d["scaling"] == scaling
    assert d["check_vs_oracle"] is True and d["zipf"]["check_vs_oracle"] is True
    # below 32 files per GPU one K3 launch every 2 submits (auto K3 period: 4 does not divide 6 steps)
    assert d["config"]["k3_period"] == 2
    assert d["window_launches"]["k1_digest_scan"] == 6 and d["window_launches"]["k3_block_md5"] == 3
    assert d["config"]["files_per_gpu"] == (4 // nproc if scaling == "strong" else 4)
    assert d["value"] > 0
    e = d["e2e"]
    assert e["check_vs_oracle"] is True and e["value"] > 0
    assert e["window_launches"]["k3_block_md5"] == e["steps"]


@pytest.mark.timeout(600)
def test_bench_configs2_full_corpus_world2():
    """configs[2] at its stated size (verdict r05 item 4): the same 64 x 128
    MiB corpus a one-GPU run hashes, strong-scaled over 2 ranks (32 files
    each, LPT), both ranks on cuda:0 sharing its HBM (each plans half of the
    free memory: ranks_per_device 2), each with the library's plan
    (hbx_plan_pipeline: lag 2, lead 3, period 1 at 32 files).  Every file of
    the last 4 batches each rank collected in the timed window, and of its
    last drained batch, is checked against the oracle."""
    d = _torchrun(2, ["bench.py", "--gpus", "2", "--steps", "8", "--warmup", "2", "--dist-backend", "gloo",
                      "--no-cpu-baseline", "--cpu-threads", "16", "--workload", "random", "--e2e-steps", "0",
                      "--no-lifetime", "--check-batches", "4"], timeout=540)
    c = d["config"]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert c["files_per_step"] == 64 and c["files_per_gpu"] == 32 and c["file_bytes"] == 128 << 20
    assert (c["join_lag"], c["scan_lead"], c["k3_period"]) == (2, 3, 1)
    assert c["pipeline_depth"] >= 16  # about half of one device's batches at 4 GiB per batch
    assert d["window_launches"]["k1_digest_scan"] == 8 and d["window_launches"]["k3_block_md5"] == 8
    assert d["check_vs_oracle"] is True and d["checked_batches_per_gpu"] == 5
    assert d["chunks_per_gpu_step"] > 900 and d["value"] > 0


def test_bench_rccl_world1_through_torchrun():
    """The driver's backend: bench.py joins an RCCL (nccl) process group with
    a device-bound init and a timeout, and its barriers and max/min reductions
    run on device tensors (world 1: RCCL cannot put two ranks on one GPU)."""
    args = [x for x in BENCH if x not in ("--dist-backend", "gloo")]
    d = _torchrun(1, args + ["--gpus", "1", "--dist-backend", "nccl", "--dist-always"])
    assert d["n_gpus"] == 1 and d["check_vs_oracle"] is True and d["zipf"]["check_vs_oracle"] is True
    assert d["window_launches"]["k3_block_md5"] * d["config"]["k3_period"] == 6 and d["value"] > 0


def test_run_sharded_engine_world2():
    d = _torchrun(2, [os.path.join("tests", "mr_sharded_worker.py")])
    assert d == {"ok": True, "files": 11, "world": 2}

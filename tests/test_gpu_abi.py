"""GPU: the C-ABI from plain C (tests/c/abi_driver.c mirrors INTEGRATION.md's
cgo stub) and the ABI's state rules, bit-exact against the oracle."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind", ["random", "constant", "tiny"])
def test_plain_c_driver_matches_oracle(oracle, tmp_path, kind):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), f"OUT={tmp_path}"], check=True)
    data = {"random": oracle.random_bytes(21 * 1024 * 1024 + 77, 91),
            "constant": np.full(17 * 1024 * 1024 + 5, 0x33, np.uint8),
            "tiny": np.frombuffer(b"hello", np.uint8)}[kind]
    f = tmp_path / "in.bin"
    data.tofile(f)
    r = subprocess.run([str(tmp_path / "abi_driver"), str(f)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert "ok" in lines
    ref = oracle.store_file(data, fast=True)
    want = [f"{int(c)} {bytes(i).hex()}" for c, i in zip(ref.cut_ends, ref.ids)]
    assert [x[5:] for x in lines if x.startswith("sync ")] == want
    assert [x[6:] for x in lines if x.startswith("async ")] == want
    assert f"content {ref.content_type} {ref.content_id.hex()}" in lines


def test_state_rules(oracle):
    """The slice is fixed while batches are pending (their launch counts were
    set at submit); a refused submit leaves nothing pending; the pipeline
    keeps going afterwards."""
    import torch
    from hashbox_amd import Engine, HbxError
    sizes = [3 << 20, 9 << 20, 131073]
    files = [oracle.random_bytes(n, 60 + i) for i, n in enumerate(sizes)]
    offs = np.array([0, 4 << 20, 14 << 20], np.uint64)
    host = np.zeros(16 << 20, np.uint8)
    for o, f in zip(offs, files):
        host[int(o):int(o) + f.size] = f
    dev = torch.from_numpy(host).to("cuda:0")
    refs = [oracle.store_file(f, fast=True) for f in files]
    with Engine(0, md5_slice=64) as e:
        e.submit_device(dev.data_ptr(), offs, sizes)
        with pytest.raises(HbxError):
            e.set_md5_slice(3)
        with pytest.raises(HbxError):  # the probe is fixed while batches are pending
            e.set_k3_probe(True)
        with pytest.raises(HbxError):  # offset not 16-byte aligned
            e.submit_device(dev.data_ptr(), offs + np.uint64(4), sizes)
        assert e.pending() == 1
        e.submit_device(dev.data_ptr(), offs, sizes)
        got = [e.wait(), e.wait()]
        assert e.pending() == 0
        e.set_md5_slice(3)  # allowed once drained
        e.set_k3_probe(True)
        e.submit_device(dev.data_ptr(), offs, sizes)
        got.append(e.wait())
        w = e.k3_wave_times()  # the probe's per-wave records of the latest K3 launch
        assert w.shape[1] == 8 and (w[:, 2] >= w[:, 0]).all()
        coop = w[w[:, 7] > 0]  # waves whose first group ran the cooperative phase: cycles advance
        assert (coop[:, 5] >= coop[:, 4]).all() and (coop[:, 6] >= (coop[:, 1] & ((1 << 56) - 1))).all()
        e.set_k3_probe(False)
        assert e.knobs()["k3_probe"] == 0
    for g in got:
        for a, r in zip(g, refs):
            assert np.array_equal(a.cut_ends, r.cut_ends) and np.array_equal(a.ids, r.ids)
            assert a.content_id == r.content_id


def test_ab_switches_need_hbx_ab(monkeypatch):
    """HBX_* A/B switches change nothing unless HBX_AB=1 (a caller's stray
    environment must not change the schedule): HBX_JOIN_LAG=3 and
    HBX_LEAN_MARKS=0 alone keep join lag 1 and lean marks."""
    from hashbox_amd import Engine
    monkeypatch.delenv("HBX_AB", raising=False)
    monkeypatch.setenv("HBX_LEAN_MARKS", "0")
    monkeypatch.setenv("HBX_JOIN_LAG", "3")
    with Engine(0) as e:
        k = e.knobs()
    assert k["ab_env"] == 0 and k["lean_marks"] == 1 and k["join_lag"] == 1, k
    monkeypatch.setenv("HBX_AB", "1")
    with Engine(0) as e:
        k = e.knobs()
    # lag 3: the next launch is preplanned on the cut stream (plan_cut 2, mode 3)
    assert k["ab_env"] == 1 and k["lean_marks"] == 0 and k["join_lag"] == 3 and k["plan_mode"] == 3, k

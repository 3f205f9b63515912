"""CPU: the C-ABI library builds, loads, and exports every symbol that
include/hbxgpu.h declares (no compute call is made without a GPU)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hbxgpu.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hbx_[a-z0-9_]+)\s*\(", src)))


def _lib_path():
    from hashbox_amd import build
    return build.build()


def test_header_declarations_nonempty():
    names = _declared()
    assert "hbx_chunk_hash" in names and "hbx_chunk_hash_device" in names and len(names) >= 15


def test_library_exports_every_declared_symbol():
    so = _lib_path()
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s+(hbx_[a-z0-9_]+)$", out, flags=re.M))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing


def test_python_binding_covers_header():
    from hashbox_amd import _lib
    assert sorted(_lib.EXPORTS) == _declared()


def test_library_loads_and_pure_helpers():
    from hashbox_amd import _lib
    L = _lib.load()
    assert L.hbx_version() >= 1
    assert L.hbx_max_chunks(0) == 1
    assert L.hbx_max_chunks(65536 * 3 + 1) == 4


def test_no_cpu_fallback_in_product():
    # the product package must not import the oracle (test infrastructure)
    pkg = os.path.join(ROOT, "hashbox_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, fn)).read()
                assert "oracle" not in txt.lower().replace("oracle-", ""), fn


def test_deflate_bound_host_only():
    from hashbox_amd import _lib
    L = _lib.load()
    assert L.hbx_deflate_bound(0) == 11
    assert L.hbx_deflate_bound(1) == 17
    assert L.hbx_deflate_bound(32768) == 11 + 32768 + 5
    assert L.hbx_deflate_bound(32769) == 11 + 32769 + 10


def test_oracle_inflate_strict_rejects_truncation():
    import zlib
    from oracle import deflate as OD
    z = zlib.compress(b"hello world" * 100)
    assert OD.inflate_strict(z) == b"hello world" * 100
    for bad in (z[:-1], z + b"\0", z[:5]):
        try:
            OD.inflate_strict(bad)
        except (ValueError, zlib.error):
            continue
        raise AssertionError("accepted a bad stream")


def test_plain_c_driver_links_and_reports_no_device(tmp_path):
    """The C-ABI from plain C, as the cgo stub of INTEGRATION.md binds it: the
    driver compiles against include/hbxgpu.h, links the in-tree library and,
    without a GPU, every call reports a status instead of aborting."""
    import pytest
    from hashbox_amd import _lib
    L = _lib.load()
    n = ctypes.c_int(0)
    if L.hbx_device_count(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is present: tests/test_gpu_abi.py runs the driver")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c"), f"OUT={tmp_path}"], check=True)
    f = tmp_path / "in.bin"
    f.write_bytes(b"hello")
    r = subprocess.run([str(tmp_path / "abi_driver"), str(f), "--expect-nodev"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().splitlines()[-1] == "nodev ok", (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("plan R=") and " lag=2 lead=3 period=4 " in r.stdout


def test_md5_argument_checks_without_device():
    """hbx_md5 rejects a null context or output before any HIP call."""
    from hashbox_amd import _lib
    L = _lib.load()
    out = (ctypes.c_uint8 * 16)()
    assert L.hbx_md5(None, None, 0, out) == -1
    assert L.hbx_md5(None, None, 0, None) == -1


def test_engine_hmac_construction_matches_reference_kats():
    """Engine.hmac / deep_hmac (core.go:51-80) is host logic around the device
    MD5; with hashlib standing in for hbx_md5 it reproduces the reference's
    HMAC rows (core_test.go:23-30, tests/golden/kat.json).  The GPU test
    test_hmac_kats_on_device_md5 runs the same rows through the device."""
    import hashlib
    import json
    from hashbox_amd.engine import Engine

    class HostMd5(Engine):
        def __init__(self):  # no device context
            pass

        def md5(self, data):
            return hashlib.md5(bytes(data)).digest()

    e = HostMd5()
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        rows = json.load(f)["hmac"]
    for r in rows:
        assert e.deep_hmac(r["depth"], r["text"].encode(), r["key"].encode()).hex() == r["out"], r
    assert e.deep_hmac(0, b"x", b"k") == bytes(16)  # DeepHmac with depth 0 returns the zero hash

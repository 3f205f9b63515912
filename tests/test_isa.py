"""CPU: invariants of the hot kernels' gfx950 code (hipcc -S, no GPU).

The product path relies on properties the compiler could silently break:
K1's loads land in LDS by DMA with hand-counted `vmcnt` waits (they hold only
if the loop has no other wait on vector memory and no scratch traffic), and
K1 and K3P run at the occupancy their design assumes (K1: four waves per
SIMD, at most 128 VGPRs; K3P: one MD5 wave and one producer wave per SIMD,
no scratch).  tools/check_asm_loads.py is the heavier reading of the same
ISA for the asm-load variants."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-o",
                    str(out), os.path.join(ROOT, "hashbox_amd", "csrc", "hbx_kernels.hip")],
                   check=True, capture_output=True, timeout=600)
    return out.read_text()


def _meta(isa, name):
    """The kernel's metadata block (amdhsa.kernels list entry)."""
    i = isa.index(f".name:           {name}\n")
    start = isa.rfind("  - .", 0, i)
    end = isa.find("  - .", i)
    blk = isa[start:end if end > 0 else len(isa)]
    get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))  # noqa: E731
    return {k: get(k) for k in ("vgpr_count", "vgpr_spill_count", "private_segment_fixed_size")}


def _body(isa, name):
    a = isa.index(f"\n{name}:")
    b = isa.index(".Lfunc_end", a)
    return [ln.split(";")[0].strip() for ln in isa[a:b].splitlines()]


def test_k1_occupancy_and_no_scratch(isa):
    m = _meta(isa, "hbx_k1_digest_scan_dma")
    assert m["vgpr_spill_count"] == 0 and m["private_segment_fixed_size"] == 0, m
    assert m["vgpr_count"] <= 128, m  # four 1024-thread waves per SIMD


def test_k1_vector_memory_waits_are_the_hand_counted_ones(isa):
    """Once K1's DMA stream has started, the only vmcnt waits are the
    hand-placed ones (4/5/6 in the loop, 0 once at the end): a compiler wait
    for all of vector memory there drains the DMA in flight (the asm wait after
    the halo used to draw one after the first two iterations' DMA, so every
    tile's first iteration waited for both; round 6 uses the builtin)."""
    body = _body(isa, "hbx_k1_digest_scan_dma")
    # the loop starts at its first hand-placed steady-state wait; before it,
    # the prologue's waits for the halo also land the first DMA (issued
    # before the halo's loads since round 6)
    first = next(i for i, ln in enumerate(body) if ln.startswith("s_waitcnt") and "vmcnt(6)" in ln)
    waits = [ln for ln in body[first:] if re.match(r"s_waitcnt .*vmcnt", ln)]
    counts = [int(re.search(r"vmcnt\((\d+)\)", w).group(1)) for w in waits]
    assert set(counts) <= {0, 4, 5, 6}, waits
    assert counts.count(0) == 1, waits


def test_k1_dma_pieces_in_one_statement(isa):
    """The four 1 KiB pieces of an iteration go out with M0 set once and the
    instruction offsets 0/1024/2048/3072 (round 6)."""
    body = _body(isa, "hbx_k1_digest_scan_dma")
    lds = [ln for ln in body if ln.startswith("buffer_load_dwordx4") and ln.endswith(" lds")]
    assert any("offset:3072" in ln for ln in lds), lds[:8]


def test_k3p_no_scratch(isa):
    m = _meta(isa, "hbx_k3p_block_md5")
    assert m["vgpr_spill_count"] == 0 and m["private_segment_fixed_size"] == 0, m
    assert m["vgpr_count"] <= 256, m  # two waves (MD5 + producer) per SIMD

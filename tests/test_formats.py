"""CPU: the library's block formats (hbx_file_entry_*, hbx_chain_block_*,
hbx_directory_block_*; hashback/hashback.go:80-214) against the oracle's
restatement (oracle/formats.py).  These entry points are pure host code, so
they run without a GPU; the device-hashed directory ids are in
tests/test_gpu_formats.py.
"""
import os
import random
import stat

import pytest

from oracle import formats as OF

F = pytest.importorskip("hashbox_amd.formats")


def _rand_entry(rng: random.Random, ctype: int) -> "F.FileEntry":
    name = bytes(rng.randrange(1, 256) for _ in range(rng.choice([0, 1, 7, 255, 300])))
    return F.FileEntry(
        file_name=name, file_size=rng.choice([0, 1, 1 << 40, -5, rng.randrange(1 << 62)]),
        file_mode=rng.randrange(1 << 32), mod_time=rng.choice([0, -1, rng.randrange(-(1 << 63), 1 << 63)]),
        reference_id=rng.randbytes(16), content_type=ctype, content_block_id=rng.randbytes(16),
        decrypt_key=rng.randbytes(16),
        file_link=rng.randbytes(rng.choice([0, 3, 4096])) if ctype == 4 else b"")


def _oracle_entry(e) -> OF.FileEntry:
    return OF.FileEntry(name=e.file_name, file_size=e.file_size, file_mode=e.file_mode, mod_time=e.mod_time,
                        reference_id=e.reference_id, content_type=e.content_type, content_id=e.content_block_id,
                        decrypt_key=e.decrypt_key, link=e.file_link)


def _normalized(e):
    """The fields FileEntry.Serialize writes for e's type."""
    return F.FileEntry(file_name=e.file_name, file_size=e.file_size, file_mode=e.file_mode, mod_time=e.mod_time,
                       reference_id=e.reference_id, content_type=e.content_type,
                       content_block_id=e.content_block_id if e.content_type in (1, 2, 3) else bytes(16),
                       decrypt_key=e.decrypt_key if e.content_type == 2 else bytes(16),
                       file_link=e.file_link if e.content_type == 4 else b"")


@pytest.mark.parametrize("ctype", [0, 1, 2, 3, 4, 7])
def test_file_entry_bytes_and_round_trip(ctype):
    rng = random.Random(ctype)
    for _ in range(20):
        e = _rand_entry(rng, ctype)
        got = F.serialize_entry(e)
        assert got == _oracle_entry(e).serialize()
        back, used = F.parse_entry(got + b"trailing")
        assert used == len(got)
        assert back == _normalized(e)


def test_file_entry_layout_by_hand():
    # hashback.go:113-132: "fent" | u32 len | name | i64 | u32 | i64 | 16 | u8 | 16 | 16
    e = F.FileEntry(file_name=b"ab", file_size=0x0102030405060708, file_mode=0x800001ED, mod_time=-2,
                    reference_id=bytes(range(16)), content_type=2, content_block_id=b"\x11" * 16,
                    decrypt_key=b"\x22" * 16)
    want = (b"fent" + b"\x00\x00\x00\x02ab" + bytes.fromhex("0102030405060708") + bytes.fromhex("800001ed")
            + b"\xff" * 7 + b"\xfe" + bytes(range(16)) + b"\x02" + b"\x11" * 16 + b"\x22" * 16)
    assert F.serialize_entry(e) == want


def test_file_entry_corrupt_and_truncated():
    e = _rand_entry(random.Random(5), 4)
    good = F.serialize_entry(e)
    with pytest.raises(F.HbxError):
        F.parse_entry(b"fenx" + good[4:])
    for cut in range(len(good)):
        with pytest.raises(F.HbxError):
            F.parse_entry(good[:cut])


@pytest.mark.parametrize("k", [0, 1, 2, 233])
def test_chain_block(k):
    rng = random.Random(k)
    ids = [rng.randbytes(16) for _ in range(k)]
    keys = [rng.randbytes(16) for _ in range(k)]
    assert F.serialize_chain_block(ids) == OF.chain_block(ids)
    blk = F.serialize_chain_block(ids, keys)
    assert blk == OF.chain_block(ids, keys)
    assert F.parse_chain_block(blk) == (ids, keys)
    with pytest.raises(F.HbxError):
        F.parse_chain_block(b"fchx" + blk[4:])
    if k:
        with pytest.raises(F.HbxError):
            F.parse_chain_block(blk[:-1])


def test_chain_block_id_is_k4_content_id(oracle):
    # the chain block hashed with links = ids is the type-3 content id (store.go:187-190)
    rng = random.Random(3)
    ids = [rng.randbytes(16) for _ in range(40)]
    assert OF.hash_data(F.serialize_chain_block(ids), ids) == oracle.py_chain_id(ids)


@pytest.mark.parametrize("n", [0, 1, 5, 300])
def test_directory_block(n):
    rng = random.Random(100 + n)
    entries = [_rand_entry(rng, rng.choice([0, 1, 2, 3, 4])) for _ in range(n)]
    data, links = F.serialize_directory_block(entries)
    odata, olinks = OF.directory_block([_oracle_entry(e) for e in entries])
    assert data == odata and links == olinks
    assert F.parse_directory_block(data) == [_normalized(e) for e in entries]
    with pytest.raises(F.HbxError):
        F.parse_directory_block(b"dblx" + data[4:])
    if n:
        with pytest.raises(F.HbxError):
            F.parse_directory_block(data[:-1])


def test_go_file_mode_matches_oracle():
    modes = [stat.S_IFREG | 0o644, stat.S_IFDIR | 0o755, stat.S_IFLNK | 0o777, stat.S_IFIFO | 0o600,
             stat.S_IFSOCK | 0o700, stat.S_IFCHR | 0o620, stat.S_IFBLK | 0o660,
             stat.S_IFREG | stat.S_ISUID | stat.S_ISGID | 0o755, stat.S_IFDIR | stat.S_ISVTX | 0o1777]
    for m in modes:
        assert F.go_file_mode(m) == OF.go_file_mode(m)
    assert F.go_file_mode(stat.S_IFDIR | 0o755) == (1 << 31) | 0o755


def test_entry_from_stat(tmp_path):
    p = tmp_path / "x"
    p.write_bytes(b"abc")
    st = os.lstat(p)
    e = F.entry_from_stat(b"x", st)
    o = OF.entry_from_stat(b"x", st)
    assert (e.file_size, e.file_mode, e.mod_time) == (o.file_size, o.file_mode, o.mod_time) == (3, OF.go_file_mode(st.st_mode), st.st_mtime_ns)

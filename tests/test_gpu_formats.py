"""GPU: directory block ids hashed on the device (hbx_directory_block_ids,
K6) and a whole tree stored through the engine (formats.store_tree), against
the oracle's restatement of storePath/storeDir/storeFile
(oracle/formats.py, oracle/hbx_oracle.c; hashback/store.go:84-397,
hashback/hashback.go:80-214).  Bit-exact.
"""
import os
import random

import numpy as np
import pytest

from oracle import formats as OF

pytestmark = pytest.mark.gpu


def _entries(rng, n):
    from hashbox_amd import formats as F
    out = []
    for _ in range(n):
        t = rng.choice([0, 1, 2, 3, 4])
        out.append(F.FileEntry(file_name=rng.randbytes(rng.randrange(1, 40)), file_size=rng.randrange(1 << 40),
                               file_mode=rng.randrange(1 << 32), mod_time=rng.randrange(1 << 62),
                               reference_id=rng.randbytes(16), content_type=t, content_block_id=rng.randbytes(16),
                               decrypt_key=rng.randbytes(16), file_link=rng.randbytes(9) if t == 4 else b""))
    return out


def _oracle_id(entries):
    return OF.directory_block_id([OF.FileEntry(name=e.file_name, file_size=e.file_size, file_mode=e.file_mode,
                                               mod_time=e.mod_time, reference_id=e.reference_id,
                                               content_type=e.content_type, content_id=e.content_block_id,
                                               decrypt_key=e.decrypt_key, link=e.file_link) for e in entries])


def test_directory_block_ids(engine):
    from hashbox_amd import formats as F
    rng = random.Random(11)
    # empty dirs, dirs with no links, one dir past 64 KiB (block spans many MD5 blocks), many small
    dirs = [[], _entries(rng, 1), [e for e in _entries(rng, 30) if e.content_type in (0, 4)], _entries(rng, 1500)]
    dirs += [_entries(rng, rng.randrange(0, 40)) for _ in range(300)]
    got = F.directory_block_ids(engine, dirs)
    want = [_oracle_id(d) for d in dirs]
    assert got == want


def _make_tree(root):
    rng = np.random.default_rng(5)
    os.makedirs(root / "a" / "b" / "c")
    os.makedirs(root / "empty")
    os.makedirs(root / "many")
    sizes = {"zero": 0, "five": 5, "min2": 131072, "min2p1": 131073, "three_mib": 3 << 20, "nine_mib": (9 << 20) + 7}
    for name, n in sizes.items():
        (root / name).write_bytes(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    (root / "a" / "b" / "c" / "deep.bin").write_bytes(rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes())
    (root / "a" / "x.txt").write_bytes(b"hello")
    for i in range(150):
        (root / "many" / f"f{i:03d}").write_bytes(rng.integers(0, 256, int(rng.integers(1, 5000)), dtype=np.uint8).tobytes())
    (root / "caf\xe9").write_bytes(b"latin")
    os.symlink("five", root / "link_to_file")
    os.symlink("a", root / "link_to_dir")
    os.mkfifo(root / "pipe")


def test_store_tree_matches_oracle(engine, oracle, tmp_path):
    from hashbox_amd import formats as F
    root = tmp_path / "tree"
    root.mkdir()
    _make_tree(root)
    ref_id = bytes(range(16))
    got = F.store_tree(engine, root, reference_id=ref_id, io_threads=4)
    odirs = {}
    want = OF.store_path(os.fsencode(root), oracle.store_file, ref_id, True, odirs)
    assert got.root.content_type == OF.TYPE_DIR == want.content_type
    assert got.root.content_block_id == want.content_id
    assert set(got.directories) == set(odirs)
    for p, (data, links, i) in odirs.items():
        assert got.directories[p] == (data, links, i), p
    assert os.fsencode(root / "pipe") in got.skipped
    # the parsed root block lists the entries the reference would write
    names = [e.file_name for e in F.parse_directory_block(got.directories[os.fsencode(root)][0])]
    assert names == sorted(names) and b"pipe" not in names and b"link_to_dir" in names

"""Hashback's per-file and per-directory block formats on
libhbxgpu, plus the tree store that ties them to the chunking engine.

Reference (fredli74/hashbox):

* ``FileEntry``, ``FileChainBlock``, ``DirectoryBlock`` and their
  ``Serialize``/``Unserialize`` — hashback/hashback.go:80-214;
* ``storeDir`` (directory block + links + id) — hashback/store.go:201-234;
* ``storePath`` (what becomes which entry type) — hashback/store.go:254-397;
* ``entryFromFileInfo`` — hashback/store.go:243-251.

Serialization runs in the library's C++ (``hbx_file_entry_*``,
``hbx_chain_block_*``, ``hbx_directory_block_*``); directory block ids are
hashed on the device in one batch per tree level (``hbx_directory_block_ids``,
kernel K6).  Errors raise :class:`HbxError`, like the reference's panics
("corrupted FileEntry" etc.).
"""
from __future__ import annotations

import ctypes
import os
import stat
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .engine import Engine, FileChunks, HbxError

TYPE_EMPTY, TYPE_DIRECTORY, TYPE_FILE_DATA, TYPE_FILE_CHAIN, TYPE_SYMLINK = 0, 1, 2, 3, 4  # hashback.go:93-99

# Go io/fs FileMode bits (the FileMode that entryFromFileInfo stores)
MODE_DIR, MODE_TEMPORARY, MODE_SYMLINK, MODE_DEVICE = 1 << 31, 1 << 28, 1 << 27, 1 << 26
MODE_NAMED_PIPE, MODE_SOCKET, MODE_SETUID, MODE_SETGID = 1 << 25, 1 << 24, 1 << 23, 1 << 22
MODE_CHAR_DEVICE, MODE_STICKY = 1 << 21, 1 << 20

_ZERO16 = bytes(16)


@dataclass
class FileEntry:
    """hashback FileEntry (hashback.go:80-90), same fields."""
    file_name: bytes
    file_size: int = 0
    file_mode: int = 0
    mod_time: int = 0
    reference_id: bytes = _ZERO16
    content_type: int = TYPE_EMPTY
    content_block_id: bytes = _ZERO16
    decrypt_key: bytes = _ZERO16
    file_link: bytes = b""

    def has_content_block_id(self) -> bool:  # hashback.go:100-102
        return self.content_type in (TYPE_DIRECTORY, TYPE_FILE_DATA, TYPE_FILE_CHAIN)


def go_file_mode(st_mode: int) -> int:
    """os.FileMode of a Linux st_mode (what Go's Lstat reports)."""
    m = st_mode & 0o777
    fmt = stat.S_IFMT(st_mode)
    m |= {stat.S_IFBLK: MODE_DEVICE, stat.S_IFCHR: MODE_DEVICE | MODE_CHAR_DEVICE, stat.S_IFDIR: MODE_DIR,
          stat.S_IFIFO: MODE_NAMED_PIPE, stat.S_IFLNK: MODE_SYMLINK, stat.S_IFSOCK: MODE_SOCKET}.get(fmt, 0)
    if st_mode & stat.S_ISGID:
        m |= MODE_SETGID
    if st_mode & stat.S_ISUID:
        m |= MODE_SETUID
    if st_mode & stat.S_ISVTX:
        m |= MODE_STICKY
    return m


def entry_from_stat(name: bytes, st: os.stat_result, reference_id: bytes = _ZERO16) -> FileEntry:
    """entryFromFileInfo (store.go:243-251)."""
    return FileEntry(file_name=name, file_size=st.st_size, file_mode=go_file_mode(st.st_mode),
                     mod_time=st.st_mtime_ns, reference_id=reference_id)


def _check(rc: int, what: str):
    if rc != 0:
        raise HbxError(f"{what}: {_lib.ERRORS.get(rc, rc)}")


_ENTRY_DTYPE = np.dtype({"names": ["name", "name_len", "file_mode", "file_size", "mod_time", "reference_id",
                                    "content_id", "decrypt_key", "link", "link_len", "content_type"],
                          "formats": ["<u8", "<u4", "<u4", "<i8", "<i8", ("u1", 16), ("u1", 16), ("u1", 16),
                                      "<u8", "<u4", "u1"],
                          "offsets": [0, 8, 12, 16, 24, 32, 48, 64, 80, 88, 92], "itemsize": 96})


def _c_entries(entries: Sequence[FileEntry]):
    """hbx_file_entry[] for many entries, built column-wise (names and links
    in one byte pool).  Returns (ctypes array view, keepalive)."""
    n = len(entries)
    rec = np.zeros(max(n, 1), _ENTRY_DTYPE)
    if n:
        names = [bytes(e.file_name) for e in entries]
        links = [bytes(e.file_link) for e in entries]
        nl = np.fromiter((len(x) for x in names), np.uint64, n)
        ll = np.fromiter((len(x) for x in links), np.uint64, n)
        pool = np.frombuffer(b"".join(names) + b"".join(links) + b"\0", np.uint8)
        base = pool.ctypes.data
        noff = np.zeros(n, np.uint64)
        noff[1:] = np.cumsum(nl[:-1])
        loff = np.zeros(n, np.uint64)
        loff[1:] = np.cumsum(ll[:-1])
        loff += np.uint64(nl.sum())
        rec["name"] = np.uint64(base) + noff
        rec["name_len"] = nl
        rec["link"] = np.uint64(base) + loff
        rec["link_len"] = ll
        rec["file_mode"] = np.fromiter((int(e.file_mode) & 0xFFFFFFFF for e in entries), np.uint32, n)
        rec["file_size"] = np.fromiter((int(e.file_size) for e in entries), np.int64, n)
        rec["mod_time"] = np.fromiter((int(e.mod_time) for e in entries), np.int64, n)
        rec["content_type"] = np.fromiter((int(e.content_type) for e in entries), np.uint8, n)
        for col, attr in (("reference_id", "reference_id"), ("content_id", "content_block_id"),
                          ("decrypt_key", "decrypt_key")):
            rec[col] = np.frombuffer(b"".join(bytes(getattr(e, attr)) for e in entries), np.uint8).reshape(n, 16)
    else:
        pool = np.zeros(1, np.uint8)
    arr = (_lib.FileEntry * max(n, 1)).from_address(rec.ctypes.data)
    return arr, (rec, pool)


def _entry_ptr(arr, i: int) -> ctypes.c_void_p:
    return ctypes.c_void_p(ctypes.addressof(arr) + 96 * i)


def _py_entry(c) -> FileEntry:
    return FileEntry(file_name=ctypes.string_at(c.name, c.name_len) if c.name_len else b"",
                     file_size=c.file_size, file_mode=c.file_mode, mod_time=c.mod_time,
                     reference_id=bytes(c.reference_id), content_type=c.content_type,
                     content_block_id=bytes(c.content_id), decrypt_key=bytes(c.decrypt_key),
                     file_link=ctypes.string_at(c.link, c.link_len) if c.link_len else b"")


def serialize_entry(e: FileEntry) -> bytes:
    """FileEntry.Serialize (hashback.go:113-132)."""
    L = _lib.load()
    arr, _keep = _c_entries([e])
    n = L.hbx_file_entry_size(ctypes.byref(arr[0]))
    out = ctypes.create_string_buffer(max(n, 1))
    used = ctypes.c_uint64()
    _check(L.hbx_file_entry_serialize(ctypes.byref(arr[0]), out, n, ctypes.byref(used)), "hbx_file_entry_serialize")
    return out.raw[:used.value]


def parse_entry(buf: bytes) -> Tuple[FileEntry, int]:
    """FileEntry.Unserialize (hashback.go:133-155): (entry, bytes used)."""
    L = _lib.load()
    src = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
    c = _lib.FileEntry()
    used = ctypes.c_uint64()
    _check(L.hbx_file_entry_parse(src, len(buf), ctypes.byref(c), ctypes.byref(used)), "corrupted FileEntry")
    return _py_entry(c), used.value


def serialize_chain_block(ids: Sequence[bytes], keys: Optional[Sequence[bytes]] = None) -> bytes:
    """FileChainBlock.Serialize (hashback.go:162-170); keys default to zero."""
    L = _lib.load()
    k = len(ids)
    idb = b"".join(bytes(i) for i in ids) or _ZERO16
    keyb = b"".join(bytes(x) for x in keys) if keys is not None else None
    out = ctypes.create_string_buffer(8 + 32 * k)
    used = ctypes.c_uint64()
    _check(L.hbx_chain_block_serialize(idb, keyb, k, out, 8 + 32 * k, ctypes.byref(used)),
           "hbx_chain_block_serialize")
    return out.raw[:used.value]


def parse_chain_block(buf: bytes) -> Tuple[List[bytes], List[bytes]]:
    """FileChainBlock.Unserialize (hashback.go:171-185): (ids, keys)."""
    L = _lib.load()
    src = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
    k = ctypes.c_uint32()
    _check(L.hbx_chain_block_parse(src, len(buf), ctypes.byref(k), None, None, 0), "corrupted FileChainBlock")
    ids = ctypes.create_string_buffer(16 * max(k.value, 1))
    keys = ctypes.create_string_buffer(16 * max(k.value, 1))
    _check(L.hbx_chain_block_parse(src, len(buf), ctypes.byref(k), ids, keys, k.value), "corrupted FileChainBlock")
    return ([ids.raw[16 * i:16 * i + 16] for i in range(k.value)],
            [keys.raw[16 * i:16 * i + 16] for i in range(k.value)])


def serialize_directory_block(entries: Sequence[FileEntry]) -> Tuple[bytes, List[bytes]]:
    """DirectoryBlock.Serialize (hashback.go:192-199) + storeDir's links
    (store.go:221-228)."""
    L = _lib.load()
    arr, _keep = _c_entries(entries)
    n = len(entries)
    size = L.hbx_directory_block_size(arr, n)
    out = ctypes.create_string_buffer(max(size, 1))
    links = ctypes.create_string_buffer(16 * max(n, 1))
    used, nl = ctypes.c_uint64(), ctypes.c_uint32()
    _check(L.hbx_directory_block_serialize(arr, n, out, size, ctypes.byref(used), links, ctypes.byref(nl)),
           "hbx_directory_block_serialize")
    return out.raw[:used.value], [links.raw[16 * i:16 * i + 16] for i in range(nl.value)]


def parse_directory_block(buf: bytes) -> List[FileEntry]:
    """DirectoryBlock.Unserialize (hashback.go:200-214)."""
    L = _lib.load()
    src = ctypes.create_string_buffer(bytes(buf), max(len(buf), 1))
    n = ctypes.c_uint32()
    _check(L.hbx_directory_block_parse(src, len(buf), None, 0, ctypes.byref(n)), "corrupted DirectoryBlock")
    arr = (_lib.FileEntry * max(n.value, 1))()
    _check(L.hbx_directory_block_parse(src, len(buf), arr, n.value, ctypes.byref(n)), "corrupted DirectoryBlock")
    return [_py_entry(arr[i]) for i in range(n.value)]


def directory_block_ids(eng: Engine, dirs: Sequence[Sequence[FileEntry]], with_blocks: bool = False):
    """storeDir's block id (store.go:230-231) for many directories at once, on
    the device (one K6 launch).  With ``with_blocks`` also returns each
    directory's (dblk bytes, links)."""
    L = _lib.load()
    flat = [e for d in dirs for e in d]
    arr, _keep = _c_entries(flat)
    counts = np.array([len(d) for d in dirs], np.uint32)
    base = np.zeros(len(dirs), np.uint64)
    if len(dirs) > 1:
        base[1:] = np.cumsum(counts[:-1], dtype=np.uint64)
    ids = np.zeros((max(len(dirs), 1), 16), np.uint8)
    eng._check(eng._L.hbx_directory_block_ids(eng._ctx, len(dirs), arr, base.ctypes.data, counts.ctypes.data,
                                              ids.ctypes.data), "hbx_directory_block_ids")
    out = [bytes(r) for r in ids[:len(dirs)]]
    if not with_blocks:
        return out
    blocks = []
    links = ctypes.create_string_buffer(16 * max(int(counts.max()) if len(dirs) else 1, 1))
    used, nl = ctypes.c_uint64(), ctypes.c_uint32()
    for d in range(len(dirs)):
        p = _entry_ptr(arr, int(base[d]))
        size = L.hbx_directory_block_size(p, int(counts[d]))
        buf = ctypes.create_string_buffer(max(size, 1))
        _check(L.hbx_directory_block_serialize(p, int(counts[d]), buf, size, ctypes.byref(used), links,
                                               ctypes.byref(nl)), "hbx_directory_block_serialize")
        blocks.append((buf.raw[:used.value], [links.raw[16 * i:16 * i + 16] for i in range(nl.value)]))
    return out, blocks


@dataclass
class TreeStore:
    """What one ``store`` of a tree produces (the Go session would send every
    block to the server): the top entry, every directory block and every
    file's chunk list."""
    root: FileEntry
    directories: Dict[bytes, Tuple[bytes, List[bytes], bytes]] = field(default_factory=dict)  # path -> (dblk, links, id)
    files: Dict[bytes, FileChunks] = field(default_factory=dict)  # path -> chunks (FileSize > 0 only)
    skipped: List[bytes] = field(default_factory=list)
    seconds: Dict[str, float] = field(default_factory=dict)  # walk, files, directories


def store_tree(eng: Engine, root, reference_id: bytes = _ZERO16, io_threads: int = 16,
               batch_bytes: int = 1 << 30) -> TreeStore:
    """storePath(root, toplevel=True) for a fresh backup (no reference cache,
    no ignore list): store.go:254-397 + storeDir (201-234) + storeFile (84-199).

    Every regular file with FileSize > 0 goes through ``Engine.store_paths`` in
    one pipelined call; the directory blocks are then hashed on the device
    level by level, deepest first (a parent's entry holds its child's id).
    """
    root = os.fsencode(os.fspath(root))
    st = os.stat(root)  # the top level follows symbolic links (store.go:263-264)
    dirs: Dict[bytes, List[Tuple[bytes, FileEntry]]] = {}
    depth: Dict[bytes, int] = {}
    file_entries: Dict[bytes, FileEntry] = {}
    out = TreeStore(root=entry_from_stat(os.path.basename(root.rstrip(b"/")) or root, st, reference_id))

    def visit(path: bytes, entry: FileEntry, info: os.stat_result, d: int) -> bool:
        m = entry.file_mode
        if m & (MODE_TEMPORARY | MODE_DEVICE | MODE_NAMED_PIPE | MODE_SOCKET):  # store.go:284-296
            out.skipped.append(path)
            return False
        if m & MODE_SYMLINK:  # store.go:297-317
            entry.content_type, entry.file_size = TYPE_SYMLINK, 0
            entry.file_link = os.readlink(path)
        elif m & MODE_DIR:  # store.go:319-334
            entry.content_type, entry.file_size = TYPE_DIRECTORY, 0
            kids = []
            with os.scandir(path) as it:
                names = sorted(e.name for e in it)  # FileInfoSlice sorts by Name() (store.go:217)
            for name in names:
                p = os.path.join(path, name)
                ki = os.lstat(p)
                ke = entry_from_stat(name, ki, reference_id)
                if visit(p, ke, ki, d + 1):
                    kids.append((p, ke))
            dirs[path] = kids
            depth[path] = d
        elif entry.file_size > 0:  # store.go:355-356
            file_entries[path] = entry
        return True

    t0 = time.perf_counter()
    if not visit(root, out.root, st, 0):
        return out
    t1 = time.perf_counter()
    paths = list(file_entries)
    if paths:
        # sizes from the walk's Lstat (FileEntry.FileSize, store.go:247)
        res = eng.store_paths(paths, io_threads=io_threads, batch_bytes=batch_bytes,
                              sizes=[file_entries[p].file_size for p in paths])
        for p, r in zip(paths, res):
            e = file_entries[p]
            e.content_type, e.content_block_id = r.content_type, r.content_id  # store.go:187-196
            out.files[p] = r
    t2 = time.perf_counter()
    by_depth: Dict[int, List[bytes]] = {}
    for p, d in depth.items():
        by_depth.setdefault(d, []).append(p)
    dir_entry = {p: e for kids in dirs.values() for p, e in kids}
    dir_entry[root] = out.root
    for d in sorted(by_depth, reverse=True):
        level = by_depth[d]
        ids, blocks = directory_block_ids(eng, [[e for _, e in dirs[p]] for p in level], with_blocks=True)
        for p, i, (data, links) in zip(level, ids, blocks):
            out.directories[p] = (data, links, i)
            dir_entry[p].content_block_id = i
    out.seconds = {"walk": t1 - t0, "files": t2 - t1, "directories": time.perf_counter() - t2}
    return out

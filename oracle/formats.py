"""CPU restatement of Hashback's per-file / per-directory block formats —
TEST INFRASTRUCTURE ONLY (imported by ``tests/`` alone; the product is the
C++ in ``hashbox_amd/csrc/hbx_formats.h`` behind ``include/hbxgpu.h``).

Follows, field by field:

* ``FileEntry.Serialize / Unserialize``  hashback/hashback.go:113-155
* ``FileChainBlock.Serialize``           hashback/hashback.go:162-170
* ``DirectoryBlock.Serialize``           hashback/hashback.go:192-199
* ``core.String``                        pkg/core/core.go:95-109 (u32 length + bytes)
* ``WriteUint8/32, WriteInt64``          pkg/core/utils.go:73-88 (big-endian)
* ``storeDir``'s links + block id        hashback/store.go:201-234, with
  ``HashData`` = MD5(BE32(#links) || links || BE32(len) || data), block.go:96-111
* Go ``os.FileMode`` bits                Go standard library ``io/fs`` (the
  layout ``entryFromFileInfo`` stores, store.go:243-251)

Parity: the reference holds no test or fixture for these formats (hashback/
has no tests), so they are pinned by source only; the block id is pinned by
the MD5 KATs like every other id.
"""
from __future__ import annotations

import hashlib
import os
import stat
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

MAGIC_ENTRY = 0x66656E74  # "fent"
MAGIC_CHAIN = 0x6663686E  # "fchn"
MAGIC_DIR = 0x64626C6B  # "dblk"

TYPE_EMPTY, TYPE_DIR, TYPE_FILE_DATA, TYPE_FILE_CHAIN, TYPE_SYMLINK = 0, 1, 2, 3, 4

# Go io/fs FileMode bits
MODE_DIR = 1 << 31
MODE_APPEND = 1 << 30
MODE_EXCLUSIVE = 1 << 29
MODE_TEMPORARY = 1 << 28
MODE_SYMLINK = 1 << 27
MODE_DEVICE = 1 << 26
MODE_NAMED_PIPE = 1 << 25
MODE_SOCKET = 1 << 24
MODE_SETUID = 1 << 23
MODE_SETGID = 1 << 22
MODE_CHAR_DEVICE = 1 << 21
MODE_STICKY = 1 << 20
MODE_IRREGULAR = 1 << 19


def go_file_mode(st_mode: int) -> int:
    """Go's os.FileMode for a POSIX st_mode (fillFileStatFromSys, os/stat_linux.go)."""
    m = st_mode & 0o777
    fmt = stat.S_IFMT(st_mode)
    if fmt == stat.S_IFBLK:
        m |= MODE_DEVICE
    elif fmt == stat.S_IFCHR:
        m |= MODE_DEVICE | MODE_CHAR_DEVICE
    elif fmt == stat.S_IFDIR:
        m |= MODE_DIR
    elif fmt == stat.S_IFIFO:
        m |= MODE_NAMED_PIPE
    elif fmt == stat.S_IFLNK:
        m |= MODE_SYMLINK
    elif fmt == stat.S_IFSOCK:
        m |= MODE_SOCKET
    if st_mode & stat.S_ISGID:
        m |= MODE_SETGID
    if st_mode & stat.S_ISUID:
        m |= MODE_SETUID
    if st_mode & stat.S_ISVTX:
        m |= MODE_STICKY
    return m


@dataclass
class FileEntry:
    name: bytes
    file_size: int = 0
    file_mode: int = 0
    mod_time: int = 0
    reference_id: bytes = bytes(16)
    content_type: int = TYPE_EMPTY
    content_id: bytes = bytes(16)
    decrypt_key: bytes = bytes(16)
    link: bytes = b""

    def has_content(self) -> bool:  # hashback.go:100-102
        return self.content_type in (TYPE_DIR, TYPE_FILE_DATA, TYPE_FILE_CHAIN)

    def serialize(self) -> bytes:  # hashback.go:113-132
        out = [struct.pack(">II", MAGIC_ENTRY, len(self.name)), self.name,
               struct.pack(">qIq", self.file_size, self.file_mode, self.mod_time),
               self.reference_id, struct.pack(">B", self.content_type)]
        if self.has_content():
            out.append(self.content_id)
        if self.content_type == TYPE_FILE_DATA:
            out.append(self.decrypt_key)
        if self.content_type == TYPE_SYMLINK:
            out += [struct.pack(">I", len(self.link)), self.link]
        return b"".join(out)

    @staticmethod
    def parse(buf: bytes, pos: int = 0) -> Tuple["FileEntry", int]:  # hashback.go:133-155
        def take(n):
            nonlocal pos
            if pos + n > len(buf):
                raise ValueError("truncated FileEntry")
            r = buf[pos:pos + n]
            pos += n
            return r
        (magic,) = struct.unpack(">I", take(4))
        if magic != MAGIC_ENTRY:
            raise ValueError("corrupted FileEntry")
        (nl,) = struct.unpack(">I", take(4))
        e = FileEntry(name=bytes(take(nl)))
        e.file_size, e.file_mode, e.mod_time = struct.unpack(">qIq", take(20))
        e.reference_id = bytes(take(16))
        (e.content_type,) = struct.unpack(">B", take(1))
        if e.has_content():
            e.content_id = bytes(take(16))
        if e.content_type == TYPE_FILE_DATA:
            e.decrypt_key = bytes(take(16))
        if e.content_type == TYPE_SYMLINK:
            (ll,) = struct.unpack(">I", take(4))
            e.link = bytes(take(ll))
        return e, pos


def chain_block(ids: Sequence[bytes], keys: Optional[Sequence[bytes]] = None) -> bytes:
    """FileChainBlock.Serialize (hashback.go:162-170)."""
    keys = keys if keys is not None else [bytes(16)] * len(ids)
    return struct.pack(">II", MAGIC_CHAIN, len(ids)) + b"".join(i + k for i, k in zip(ids, keys))


def directory_block(entries: Sequence[FileEntry]) -> Tuple[bytes, List[bytes]]:
    """DirectoryBlock.Serialize (hashback.go:192-199) and storeDir's links
    (store.go:221-228)."""
    data = struct.pack(">II", MAGIC_DIR, len(entries)) + b"".join(e.serialize() for e in entries)
    links = [e.content_id for e in entries if e.has_content()]
    return data, links


def hash_data(data: bytes, links: Sequence[bytes] = ()) -> bytes:
    """HashboxBlock.HashData (block.go:96-111)."""
    h = hashlib.md5()
    h.update(struct.pack(">I", len(links)))
    for link in links:
        h.update(link)
    h.update(struct.pack(">I", len(data)))
    h.update(data)
    return h.digest()


def directory_block_id(entries: Sequence[FileEntry]) -> bytes:
    data, links = directory_block(entries)
    return hash_data(data, links)


def entry_from_stat(name: bytes, st: os.stat_result, reference_id: bytes = bytes(16)) -> FileEntry:
    """entryFromFileInfo (store.go:243-251)."""
    return FileEntry(name=name, file_size=st.st_size, file_mode=go_file_mode(st.st_mode),
                     mod_time=st.st_mtime_ns, reference_id=reference_id)


def store_path(path: bytes, store_file, reference_id: bytes = bytes(16), toplevel: bool = True,
               dirs: Optional[dict] = None) -> Optional[FileEntry]:
    """storePath (store.go:254-397) + storeDir (store.go:201-234) for a fresh
    backup (no reference cache, no ignore list), recursing exactly as the
    reference does.  ``store_file(bytes) -> oracle FileResult`` is storeFile.
    ``dirs`` (if given) collects path -> (dblk bytes, links, id)."""
    st = os.stat(path) if toplevel else os.lstat(path)
    e = entry_from_stat(os.path.basename(path.rstrip(b"/")) or path, st, reference_id)
    m = e.file_mode
    if m & (MODE_TEMPORARY | MODE_DEVICE | MODE_NAMED_PIPE | MODE_SOCKET):
        return None
    if m & MODE_SYMLINK:
        e.content_type, e.file_size, e.link = TYPE_SYMLINK, 0, os.readlink(path)
    elif m & MODE_DIR:
        e.content_type, e.file_size = TYPE_DIR, 0
        with os.scandir(path) as it:
            names = sorted(x.name for x in it)
        kids = [store_path(os.path.join(path, n), store_file, reference_id, False, dirs) for n in names]
        kids = [k for k in kids if k is not None]
        data, links = directory_block(kids)
        e.content_id = hash_data(data, links)
        if dirs is not None:
            dirs[path] = (data, links, e.content_id)
    elif e.file_size > 0:
        with open(path, "rb") as fh:
            r = store_file(fh.read())
        e.content_type, e.content_id = r.content_type, r.content_id
    return e

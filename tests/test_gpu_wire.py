"""GPU: the client's send path end to end over a socket.
Files on disk -> hbx_store_paths_zcb (chunk ids + device zlib per batch) ->
allo / READ / writ / ACKN through the product's wire encoders and parser ->
an in-process sink restating server.go:160-202 that re-verifies every
written block (UncompressData + HashData, server.go:182) and answers
already-stored blocks with ACKN (dedup)."""
import ctypes
import socket
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_store_paths_to_loopback_sink(engine, oracle, tmp_path):
    from hashbox_amd import _lib
    from oracle import wire as OW
    L = _lib.load()
    rng = np.random.default_rng(31)
    paths, datas = [], []
    for i in range(36):
        n = int(rng.integers(1, 20 << 20)) if i % 9 else int(rng.integers(9 << 20, 17 << 20))
        if i in (7, 19, 30):  # duplicates of earlier files: their chunks dedup at the sink
            d = datas[i - 5]
        elif i % 4 == 3:  # compressible
            d = (rng.integers(0, 256, 3000, dtype=np.uint8).tobytes() * (n // 3000 + 1))[:n]
        else:
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        p = tmp_path / f"w{i:02d}"
        p.write_bytes(d)
        paths.append(p)
        datas.append(d)
    preseed = [bytes(x) for x in oracle.store_file(np.frombuffer(datas[2], np.uint8), fast=True).ids]

    cli, srv = socket.socketpair()
    sink = OW.LoopbackSink(srv, preseed).start()
    lock = threading.Lock()
    pending = {}  # num -> (id, zlib stream)
    acked, errors = [], []
    done = threading.Event()
    state = {"num": 0, "sent": 0}

    def send(b):
        with lock:
            cli.sendall(b)

    def receiver():
        buf = b""
        while True:
            chunk = cli.recv(1 << 16)
            if not chunk:
                return
            buf += chunk
            while True:
                m = _lib.WireMsg()
                src = ctypes.create_string_buffer(buf, max(len(buf), 1))
                rc = L.hbx_wire_parse(src, len(buf), ctypes.byref(m))
                if rc == -3:
                    break
                assert rc == 0
                if m.type == OW.READ & OW.SERVER_MASK:
                    bid, z = pending[m.num]
                    hdr = ctypes.create_string_buffer(64)
                    used = ctypes.c_uint64()
                    assert L.hbx_wire_encode_block_header(m.num, OW.WRITE, bid, None, 0, OW.ZLIB, len(z), hdr, 64,
                                                          ctypes.byref(used)) == 0
                    send(hdr.raw[:used.value] + z)
                elif m.type == OW.ACKNOWLEDGE & OW.SERVER_MASK:
                    assert bytes(m.id) == pending[m.num][0]
                    acked.append(bytes(m.id))
                elif m.type == OW.ERROR & OW.SERVER_MASK:
                    errors.append(ctypes.string_at(m.data, m.data_len))
                elif m.type == OW.GOODBYE & OW.SERVER_MASK:
                    done.set()
                    return
                buf = buf[m.total_len:]

    rt = threading.Thread(target=receiver, daemon=True)
    rt.start()

    def on_files(first, files):  # StoreBlock for every chunk as soon as its batch is stored
        for f in files:
            for bid, z in zip(f.ids, f.zstreams):
                num = state["num"]
                state["num"] = (num + 1) & 0xFFFF
                pending[num] = (bytes(bid), bytes(z))
                out = (ctypes.c_uint8 * 22)()
                assert L.hbx_wire_encode_id(num, OW.ALLOCATE, bytes(bid), out) == 0
                send(bytes(out))
                state["sent"] += 1

    res = engine.store_paths(paths, io_threads=4, batch_bytes=64 << 20, compress=True, on_files=on_files)
    total = sum(r.n_chunks for r in res)
    assert state["sent"] == total and total < 65536
    for _ in range(600):
        if len(acked) + len(errors) >= total:
            break
        threading.Event().wait(0.05)
    send(OW.header(0, OW.GOODBYE))
    assert done.wait(30)
    cli.close()
    assert errors == [] and sink.failed == 0
    assert len(acked) == total  # every allo ends in exactly one ACKN
    ids_all = [bytes(x) for r in res for x in r.ids]
    assert sorted(acked) == sorted(ids_all)
    assert sink.verified == sink.reads  # every READ was answered by a writ that verified
    assert sink.acked_allocs >= len(preseed)  # dedup: the preseeded file's chunks were never sent
    assert sink.verified <= len(set(ids_all) - set(preseed)) + 3 * 8  # racing duplicates may both be written
    for d, r in zip(datas, res):  # the ids sent are the reference's ids
        ref = oracle.store_file(np.frombuffer(d, np.uint8), fast=True)
        assert np.array_equal(r.cut_ends, ref.cut_ends) and np.array_equal(r.ids, ref.ids)

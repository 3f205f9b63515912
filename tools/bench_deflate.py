#!/usr/bin/env python3
"""Device zlib block compression (HashboxBlock.CompressData) on
the chunks the engine cuts, device-resident:

  random   the configs[1] batch: 64 x 128 MiB uniform random, every chunk
  text     1 GiB of Zipf-distributed words (a 64 MiB generated text tiled),
           every chunk

Per corpus: device time of hbx_deflate_blocks_device (all chunks of the
batch in one call: K7a + K7s + K7b), GB/s of input, compressed / input ratio,
and beside it CPython zlib level 6 (Go's DefaultCompression stand-in,
oracle/deflate.py) on 16 threads over a sample of the same chunks.  Every
stream of a sample is inflated by the oracle and compared (round trip).

Run on the GPU box: python tools/bench_deflate.py     (prints one JSON line)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def text_corpus(nbytes, seed):
    rng = np.random.default_rng(seed)
    vocab = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(2, 11, 5000)]
    ids = rng.zipf(1.2, 12_000_000) % len(vocab)
    base = b" ".join(vocab[i] for i in ids)[: 64 << 20]
    reps = (nbytes + len(base) - 1) // len(base)
    return np.frombuffer((base * reps)[:nbytes], np.uint8)


def run_corpus(eng, torch, name, host_or_dev, file_bytes, nfiles, sample, threads):
    from oracle import deflate as OD
    if isinstance(host_or_dev, np.ndarray):
        arena = torch.empty(host_or_dev.size + 65536, dtype=torch.uint8, device="cuda:0")
        arena[: host_or_dev.size].copy_(torch.from_numpy(host_or_dev))
    else:
        arena = host_or_dev
    torch.cuda.synchronize()
    offs = np.arange(nfiles, dtype=np.uint64) * np.uint64(file_bytes)
    res = eng.chunk_hash_device(arena.data_ptr(), offs, [file_bytes] * nfiles)
    c_off, c_len = [], []
    for f, r in enumerate(res):
        starts, ends = r.chunk_bounds()
        c_off += list(offs[f] + starts)
        c_len += list(ends - starts)
    c_off = np.array(c_off, np.uint64)
    c_len = np.array(c_len, np.uint64)
    caps = np.array([eng.deflate_bound(int(n)) for n in c_len], np.uint64)
    o_off = np.zeros_like(caps)
    o_off[1:] = np.cumsum(caps[:-1])
    out = torch.empty(int(caps.sum()) + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    eng.deflate_blocks_device(arena.data_ptr(), c_off[:8], c_len[:8], out.data_ptr(), o_off[:8], caps[:8])  # warm-up
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        lens = eng.deflate_blocks_device(arena.data_ptr(), c_off, c_len, out.data_ptr(), o_off, caps)
        times.append(time.perf_counter() - t0)
    t = min(times)
    total_in = int(c_len.sum())
    total_out = int(lens.sum())
    # round trip + CPU zlib -6 on a sample of chunks
    rng = np.random.default_rng(3)
    pick = np.sort(rng.choice(c_off.size, min(sample, c_off.size), replace=False))
    host_in = arena[: int(offs[-1]) + file_bytes].cpu().numpy()
    host_out = out.cpu().numpy()
    blocks = [host_in[int(c_off[i]): int(c_off[i] + c_len[i])].tobytes() for i in pick]
    bad = 0
    for i, b in zip(pick, blocks):
        z = host_out[int(o_off[i]): int(o_off[i] + lens[i])].tobytes()
        bad += OD.inflate_strict(z) != b
    t0 = time.perf_counter()
    ref = OD.compress_ref_mt(blocks, threads)
    t_cpu = time.perf_counter() - t0
    s_in = sum(len(b) for b in blocks)
    s_gpu = sum(int(lens[i]) for i in pick)
    # device inflate of the device's own streams (every chunk), checked on the sample
    icap = c_len.copy()
    i_off = np.zeros_like(icap)
    i_off[1:] = np.cumsum(icap[:-1])
    back = torch.empty(int(icap.sum()) + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ilen, ist = eng.inflate_blocks_device(out.data_ptr(), o_off, lens, back.data_ptr(), i_off, icap)
    t_inf = time.perf_counter() - t0
    ib = back.cpu().numpy()
    ibad = int((ist != 0).sum()) + sum(ib[int(i_off[i]):int(i_off[i] + ilen[i])].tobytes() != b
                                       for i, b in zip(pick, blocks))
    t0 = time.perf_counter()
    OD.inflate_mt([host_out[int(o_off[i]): int(o_off[i] + lens[i])].tobytes() for i in pick], threads)
    t_cinf = time.perf_counter() - t0
    zl = inflate_zlib6(eng, torch, host_in, c_off, c_len, threads) if name == "text" else None
    out = {
        "inflate_device": {"seconds": round(t_inf, 4), "gbs_out": round(total_in / t_inf / 1e9, 2),
                           "streams": int(c_off.size), "failures_or_mismatches": ibad,
                           "cpu_zlib_inflate_gbs_out": round(s_in / t_cinf / 1e9, 3), "cpu_threads": threads},
        "chunks": int(c_off.size), "bytes_in": total_in, "bytes_out": total_out,
        "ratio": round(total_out / total_in, 4), "seconds": round(t, 4),
        "gbs": round(total_in / t / 1e9, 2), "gibs": round(total_in / t / 2**30, 2),
        "sample_chunks": int(pick.size), "sample_roundtrip_mismatches": int(bad),
        "sample_ratio_gpu": round(s_gpu / s_in, 4),
        "cpu_zlib6": {"threads": threads, "ratio": round(sum(map(len, ref)) / s_in, 4),
                      "gbs": round(s_in / t_cpu / 1e9, 3), "sample_bytes": s_in},
    }
    if zl is not None:
        out["inflate_zlib6_device"] = zl
    return out


def inflate_zlib6(eng, torch, host_in, c_off, c_len, threads):
    """Every chunk of the corpus compressed by CPython zlib -6 (the stand-in
    for Go's compress/zlib DefaultCompression, block.go:216), inflated on the
    device in one call (K8: long streams split into regions, K8s) and by
    CPython on `threads`; every stream checked."""
    from oracle import deflate as OD
    blocks = [host_in[int(o): int(o + n)].tobytes() for o, n in zip(c_off, c_len)]
    zs = OD.compress_ref_mt(blocks, threads)
    io = np.zeros(len(zs), np.uint64)
    io[1:] = np.cumsum([(len(z) + 15) // 16 * 16 for z in zs[:-1]])
    host = np.zeros(int(io[-1]) + len(zs[-1]) + 64, np.uint8)
    for o, z in zip(io, zs):
        host[int(o):int(o) + len(z)] = np.frombuffer(z, np.uint8)
    d_in = torch.from_numpy(host).to("cuda:0")
    caps = np.asarray(c_len, np.uint64)
    oo = np.zeros_like(caps)
    oo[1:] = np.cumsum(caps[:-1])
    d_out = torch.empty(int(caps.sum()) + 64, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    k0 = eng.knobs()
    times = []
    for _ in range(2):
        t0 = time.perf_counter()
        ol, st = eng.inflate_blocks_device(d_in.data_ptr(), io, [len(z) for z in zs], d_out.data_ptr(), oo, caps)
        times.append(time.perf_counter() - t0)
    k1 = eng.knobs()
    back = d_out.cpu().numpy()
    bad = int((st != 0).sum()) + sum(back[int(o):int(o) + len(b)].tobytes() != b for o, b in zip(oo, blocks))
    t0 = time.perf_counter()
    OD.inflate_mt(zs, threads)
    t_cpu = time.perf_counter() - t0
    total = int(caps.sum())
    return {"streams": len(zs), "bytes_out": total, "compressed_bytes": int(sum(map(len, zs))),
            "seconds": round(min(times), 4), "gbs_out": round(total / min(times) / 1e9, 2),
            "failures_or_mismatches": bad,
            "split_streams": (k1["k8_split_streams"] - k0["k8_split_streams"]) // 2,
            "split_fallbacks": (k1["k8_split_fallbacks"] - k0["k8_split_fallbacks"]) // 2,
            "cpu_zlib_inflate": {"threads": threads, "gbs_out": round(total / t_cpu / 1e9, 3)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--file-mib", type=int, default=128)
    ap.add_argument("--sample", type=int, default=64)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    from hashbox_amd import Engine
    fb = a.file_mib << 20
    eng = Engine(0)
    out = {"workload": "device zlib (K7) over every chunk of a batch, device-resident"}
    try:
        g = torch.Generator(device="cuda:0")
        g.manual_seed(1)
        arena = torch.empty(a.files * fb + 65536, dtype=torch.uint8, device="cuda:0")
        arena.random_(0, 256, generator=g)
        out["random"] = run_corpus(eng, torch, "random", arena, fb, a.files, a.sample, a.threads)
        del arena
        torch.cuda.empty_cache()
        txt = text_corpus(8 * fb, 5)
        out["text"] = run_corpus(eng, torch, "text", txt, fb, 8, a.sample, a.threads)
        out["inflate_many_small"] = inflate_many(eng, torch, txt, a.threads)
    finally:
        eng.close()
    print(json.dumps(out), flush=True)


def inflate_many(eng, torch, txt, threads, n=65536, size=16384):
    """Many small zlib -6 streams (the stand-in for Go-compressed stored
    blocks): K8 with one lane per stream vs CPython zlib on `threads`."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    from oracle import deflate as OD
    rng = np.random.default_rng(9)
    starts = rng.integers(0, txt.size - size, n)
    raw = [txt[int(s0):int(s0) + size].tobytes() for s0 in starts]
    with ThreadPoolExecutor(threads) as ex:
        zs = list(ex.map(lambda b: zlib.compress(b, 6), raw))
    io = np.zeros(n, np.uint64)
    io[1:] = np.cumsum([(len(z) + 15) // 16 * 16 for z in zs[:-1]])
    host = np.zeros(int(io[-1]) + len(zs[-1]) + 64, np.uint8)
    for o, z in zip(io, zs):
        host[int(o):int(o) + len(z)] = np.frombuffer(z, np.uint8)
    d_in = torch.from_numpy(host).to("cuda:0")
    oo = np.arange(n, dtype=np.uint64) * np.uint64(size)
    d_out = torch.empty(n * size + 64, dtype=torch.uint8, device="cuda:0")
    caps = np.full(n, size, np.uint64)
    torch.cuda.synchronize()
    eng.inflate_blocks_device(d_in.data_ptr(), io[:64], [len(z) for z in zs[:64]], d_out.data_ptr(), oo[:64], caps[:64])
    t0 = time.perf_counter()
    ol, st = eng.inflate_blocks_device(d_in.data_ptr(), io, [len(z) for z in zs], d_out.data_ptr(), oo, caps)
    t = time.perf_counter() - t0
    back = d_out.cpu().numpy()
    bad = int((st != 0).sum()) + sum(back[i * size:(i + 1) * size].tobytes() != raw[i] for i in range(0, n, 97))
    t0 = time.perf_counter()
    OD.inflate_mt(zs, threads)
    t_cpu = time.perf_counter() - t0
    return {"streams": n, "stream_bytes": size, "compressed_bytes": int(sum(map(len, zs))),
            "seconds": round(t, 4), "gbs_out": round(n * size / t / 1e9, 2), "failures_or_mismatches": bad,
            "cpu_zlib_inflate": {"threads": threads, "gbs_out": round(n * size / t_cpu / 1e9, 3)}}


if __name__ == "__main__":
    main()

"""Synthetic device-resident inputs for bench.py and the GPU tests (not part
of the product path).

* configs[1]: batches of 64 x 128 MiB uniform random bytes.
* configs[3]: a Zipf-duplicated corpus (~50 % repeat content): segments of
  64 KiB-4 MiB; each draw takes a fresh random segment with probability 1/2,
  otherwise re-uses an earlier one chosen by Zipf(1.1) rank (rank 1 = the
  first segment drawn).  Repeats may cross batches: the corpus is one stream
  cut into the resident batches.  Same scheme as tools/validate_config4.py.

Everything is generated on the device (torch), so a bench fills 260+ GiB of
HBM in seconds; a host copy is taken only to run the CPU oracle.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

SEG_MIN = 64 * 1024
SEG_MAX = 4 * 1024 * 1024


def pack_layout(lens: Sequence[int], align: int = 256, slack: int = 65536) -> Tuple[np.ndarray, int]:
    """Offsets of files packed into one arena (256-B aligned) and the bytes to
    allocate (the engine reads up to 63 bytes past a file, K1 a halo)."""
    offs = np.zeros(len(lens), np.uint64)
    pos = 0
    for i, n in enumerate(lens):
        offs[i] = pos
        pos += (int(n) + align - 1) // align * align
    return offs, pos + slack


def random_arenas(count: int, total: int, seed: int, device, single: bool = False) -> list:
    """`count` distinct arenas of `total` uniform random bytes (with `single`:
    views of one allocation, 2 MiB-aligned)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = []
    if single:
        step = (total + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        big = torch.empty(step * count, dtype=torch.uint8, device=device)
        out = [big[i * step:i * step + total] for i in range(count)]
        for t in out:
            t.random_(0, 256, generator=g)
        return out
    for _ in range(count):
        t = torch.empty(total, dtype=torch.uint8, device=device)
        t.random_(0, 256, generator=g)
        out.append(t)
    return out


def corpus_seed(seed: int, batch: int, file: int) -> int:
    """Generator seed of job file `file` of resident batch `batch`."""
    return (seed * 1_000_003 + batch * 65_537 + file) & 0x7FFFFFFFFFFFFFFF


def fill_batch(arena, batch: int, offs: Sequence[int], lens: Sequence[int], file_ids: Sequence[int],
               seed: int) -> None:
    """Write the files of one resident batch: file k (job file file_ids[k])
    gets uniform random bytes from its own generator, seeded by (seed, batch,
    job file), so a job file's bytes do not depend on which rank holds it or
    how many ranks share the step (strong scaling splits ONE corpus).  The
    padding between files is left as allocated: no result depends on it."""
    import torch
    g = torch.Generator(device=arena.device)
    for o, n, j in zip(offs, lens, file_ids):
        g.manual_seed(corpus_seed(seed, batch, int(j)))
        arena[int(o):int(o) + int(n)].random_(0, 256, generator=g)


def corpus_arenas(count: int, total: int, offs: Sequence[int], lens: Sequence[int], file_ids: Sequence[int],
                  seed: int, device, single: bool = False) -> list:
    """`count` resident batches of the job corpus (fill_batch), each in an
    arena of `total` bytes (with `single`: views of one allocation, 2 MiB-aligned)."""
    import torch
    if single:
        step = (total + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        big = torch.empty(step * count, dtype=torch.uint8, device=device)
        out = [big[i * step:i * step + total] for i in range(count)]
    else:
        out = [torch.empty(total, dtype=torch.uint8, device=device) for _ in range(count)]
    for b, t in enumerate(out):
        fill_batch(t, b, offs, lens, file_ids, seed)
    return out


def zipf_fill(arenas: list, used: int, seed: int, fresh_p: float = 0.5, a: float = 1.1) -> float:
    """Overwrite bytes [0, used) of every arena with one Zipf-duplicated
    stream (configs[3] scheme).  Returns the repeat fraction: bytes of
    second and later occurrences / all bytes."""
    import torch
    g = np.random.Generator(np.random.PCG64(seed))
    tg = torch.Generator(device=arenas[0].device)
    tg.manual_seed(seed)
    segs: List[Tuple[int, int, int]] = []  # (arena, offset, size) of first occurrences
    repeat = 0
    for ai, arena in enumerate(arenas):
        pos = 0
        while pos < used:
            if not segs or g.random() < fresh_p:
                size = min(int(g.integers(SEG_MIN, SEG_MAX + 1)), used - pos)
                arena[pos:pos + size].random_(0, 256, generator=tg)
                segs.append((ai, pos, size))
            else:
                r = int(min(g.zipf(a), len(segs))) - 1
                sa, so, size = segs[r]
                size = min(size, used - pos)
                arena[pos:pos + size].copy_(arenas[sa][so:so + size])
                repeat += size
            pos += size
    torch.cuda.synchronize(arenas[0].device)
    return repeat / (used * len(arenas))

"""File -> GPU assignment.  Files are independent: each GPU
chunks and hashes its own files; no collective is on the data path."""
from __future__ import annotations

import heapq
from typing import List, Sequence


def lpt_assign(lens: Sequence[int], n_gpus: int) -> List[List[int]]:
    """Longest-processing-time-first: biggest file to the least-loaded GPU.
    Returns per-GPU lists of file indices (each list in ascending order)."""
    if n_gpus < 1:
        raise ValueError("n_gpus must be >= 1")
    heap = [(0, g) for g in range(n_gpus)]
    out: List[List[int]] = [[] for _ in range(n_gpus)]
    for i in sorted(range(len(lens)), key=lambda i: (-int(lens[i]), i)):
        load, g = heapq.heappop(heap)
        out[g].append(i)
        heapq.heappush(heap, (load + int(lens[i]), g))
    return [sorted(x) for x in out]

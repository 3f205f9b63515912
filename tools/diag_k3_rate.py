"""Dev diagnostic: per-chain MD5 rate with exact 8 MiB chunks (constant
bytes cut at exactly MAX), alone vs many concurrent waves."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from hashbox_amd import Engine, pack_arena_layout

MAXB = 8 * 1024 * 1024
e = Engine(0)
for nfiles in [1, 33, 64, 128]:
    lens = [MAXB + 1] * nfiles
    offs, total = pack_arena_layout(lens)
    arena = torch.full((total,), 0x5A, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    for _ in range(2):
        r = e.chunk_hash_device(arena.data_ptr(), offs, lens)
    st = e.stage_times()
    blocks = (MAXB + 8) // 64
    print(f"files={nfiles:4d} chunks/file={r[0].n_chunks} K3={st[2]:.2f} ms  "
          f"ns/block={st[2] * 1e6 / blocks:.1f}  stages={st.round(3)}", flush=True)

// EXPERIMENT (not built): "wave mode" block MD5 — one chunk per wave.
// v1 (W from LDS each group) and v2 (below: W for the next block read one
// block early into a second register set, chain = 4 VALU/step, ~315 instrs
// per 64-B block against ~373 in lane mode) both measured 633-637 ns per
// block on exact 8 MiB chains — the same as lane mode — and v2 ran the
// 64 x 128 MiB batch in 136 ms against 88 ms in lane mode.  Conclusion: the
// MD5 chain is bound by its 4 dependent VALU per step (~6 cycles each at
// 2.4 GHz), not by issue; lane mode already packs 64 chains into one
// instruction stream at that bound.  See DESIGN.md "K3".
// Depends on hbx_kernels.hip helpers (HBX_F.., rotl, msg_word, md5_init,
// make_rsrc_u, u32x4).
// ------------------------------------------------------ K3 wave mode ----
// One chunk per wave.  The 64 lanes build the step words of a future block in
// parallel (lane i: W_i = M[g(i)] + T_i) into an LDS slot; the next block's
// 64 words are read into a second register set one block ahead; the serial
// chain then costs 4 VALU per step (bitop3, add3, alignbit, add) with no
// memory wait, against ~5.8 in lane mode.  Used for the longest chunks (the
// batch's critical path), at most 2 such waves per SIMD.
#define HBX_VREG4(w) asm("" : "+v"(w))
#define HBX_STEPW(FN, a, b, c, d, w, s) a = (b) + rotl((a) + (FN(b, c, d)) + (w), s)

__constant__ uint32_t kMd5T[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u,
    0xfd469501u, 0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u,
    0xa679438eu, 0x49b40821u, 0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du,
    0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u, 0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu,
    0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au, 0xfffa3942u, 0x8771f681u, 0x6d9d6122u,
    0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u, 0x289b7ec6u, 0xeaa127fau,
    0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u, 0xf4292244u,
    0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu,
    0xeb86d391u};

// 16 x u32x4 = the 64 step words of one block, replicated in every lane.
struct WBlock {
  u32x4 w[16];
};

__device__ __forceinline__ void wblock_read(WBlock& W, const uint32_t* slot) {
  const u32x4* p = reinterpret_cast<const u32x4*>(slot);
#pragma unroll
  for (int i = 0; i < 16; i++) W.w[i] = p[i];
}

// Make a block's words opaque VGPR values (keeps the chain on the VALU) and
// force their LDS reads complete — call it BEFORE issuing the next block's
// reads: the in-order lgkm counter saturates at 15 outstanding reads.
__device__ __forceinline__ void wblock_pin(WBlock& W) {
#pragma unroll
  for (int i = 0; i < 16; i++) HBX_VREG4(W.w[i]);
}

__device__ __forceinline__ void md5_compress_wb(uint32_t (&h)[4], const WBlock& W) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
#define HBX_R4(FN, q, s0, s1, s2, s3)                 \
  HBX_STEPW(FN, a, b, c, d, W.w[q].x, s0);            \
  HBX_STEPW(FN, d, a, b, c, W.w[q].y, s1);            \
  HBX_STEPW(FN, c, d, a, b, W.w[q].z, s2);            \
  HBX_STEPW(FN, b, c, d, a, W.w[q].w, s3);
  HBX_R4(HBX_F, 0, 7, 12, 17, 22) HBX_R4(HBX_F, 1, 7, 12, 17, 22)
  HBX_R4(HBX_F, 2, 7, 12, 17, 22) HBX_R4(HBX_F, 3, 7, 12, 17, 22)
  HBX_R4(HBX_G, 4, 5, 9, 14, 20) HBX_R4(HBX_G, 5, 5, 9, 14, 20)
  HBX_R4(HBX_G, 6, 5, 9, 14, 20) HBX_R4(HBX_G, 7, 5, 9, 14, 20)
  HBX_R4(HBX_H, 8, 4, 11, 16, 23) HBX_R4(HBX_H, 9, 4, 11, 16, 23)
  HBX_R4(HBX_H, 10, 4, 11, 16, 23) HBX_R4(HBX_H, 11, 4, 11, 16, 23)
  HBX_R4(HBX_I, 12, 6, 10, 15, 21) HBX_R4(HBX_I, 13, 6, 10, 15, 21)
  HBX_R4(HBX_I, 14, 6, 10, 15, 21) HBX_R4(HBX_I, 15, 6, 10, 15, 21)
#undef HBX_R4
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
}

// MD5(BE32(0) || BE32(len) || chunk) by one whole wave; result in every lane.
// wring: this wave's 2 x 64 u32 LDS slots.
__device__ void md5_chunk_wave(const uint8_t* c, uint32_t len, uint32_t* __restrict__ wring,
                               uint32_t (&h)[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gi = lane < 16 ? lane
                    : lane < 32 ? ((5u * lane + 1u) & 15u)
                    : lane < 48 ? ((3u * lane + 5u) & 15u)
                                : ((7u * lane) & 15u);
  const uint32_t Ti = kMd5T[lane];
  const uint64_t cp = reinterpret_cast<uint64_t>(c);
  const uint32_t sh = (uint32_t)cp & 3u;
  const __amdgpu_buffer_rsrc_t rs =
      make_rsrc_u(reinterpret_cast<const void*>(cp - sh), (sh + len + 64u + 15u) & ~15u);
  const uint32_t T = len + 8u;
  const uint32_t nb = (T + 9u + 63u) >> 6;  // blocks incl. padding
  const uint64_t bits = (uint64_t)T * 8ull;
  // raw dword pair around message word g(i) of block bb: R[16bb+gi-2..-1]
  auto raw_load = [&](uint32_t bb) -> uint2 {
    const uint32_t off = 4u * (16u * bb + gi) - 8u;  // wraps below 0 -> out of range -> 0
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0u, 0));
  };
  auto produce = [&](uint32_t bb, uint2 raw, uint32_t slot) {
    uint32_t m = msg_word(16u * bb + gi, raw.x, raw.y, sh, len);
    if (bb + 1u == nb) {
      if (gi == 14u) m = (uint32_t)bits;
      if (gi == 15u) m = (uint32_t)(bits >> 32);
    }
    wring[slot * 64u + lane] = m + Ti;
  };
  md5_init(h);
  uint2 ring[4];
#pragma unroll
  for (int r = 0; r < 4; r++) ring[r] = raw_load((uint32_t)r);
  produce(0u, ring[0], 0u);
  ring[0] = raw_load(4u);
  if (nb > 1u) {
    produce(1u, ring[1], 1u);
    ring[1] = raw_load(5u);
  }
  WBlock Wa, Wb;
  wblock_read(Wa, wring);
  // invariant at the top: Wa = W(b); LDS slot (b+1)&1 holds W(b+1);
  // ring[k&3] holds the raw words of block k for k in b+2 .. b+5
  for (uint32_t b = 0; b < nb; b += 2u) {  // wave-uniform
    wblock_pin(Wa);
    __builtin_amdgcn_sched_barrier(0);
    if (b + 1u < nb) wblock_read(Wb, wring + 64u);
    if (b + 2u < nb) {
      produce(b + 2u, ring[2], 0u);
      ring[2] = raw_load(b + 6u);
    }
    __builtin_amdgcn_sched_barrier(0);
    md5_compress_wb(h, Wa);
    if (b + 1u < nb) {
      wblock_pin(Wb);
      __builtin_amdgcn_sched_barrier(0);
      if (b + 2u < nb) wblock_read(Wa, wring);
      if (b + 3u < nb) {
        produce(b + 3u, ring[3], 1u);
        ring[3] = raw_load(b + 7u);
      }
      __builtin_amdgcn_sched_barrier(0);
      md5_compress_wb(h, Wb);
    }
    // rotate the raw ring by two blocks
    const uint2 t0 = ring[0], t1 = ring[1];
    ring[0] = ring[2];
    ring[1] = ring[3];
    ring[2] = t0;
    ring[3] = t1;
  }
}


// EXPERIMENT (not built): "wave mode" block MD5 — one chunk per wave, the 64
// lanes precompute W_i = M[g(i)] + T_i for the next block into LDS so the
// serial chain needs 4 VALU per step instead of 5.  Measured on MI355X
// (round 1): 85 ms for a ~8 MiB chunk vs 73 ms in lane mode, and 1.7x slower
// than lane mode on the 64 x 128 MiB batch (many single-chain waves share
// SIMDs).  Kept for reference; see DESIGN.md "K3".
// Depends on hbx_kernels.hip helpers (HBX_F.., rotl, msg_word, md5_init).
// The step words are wave-uniform (LDS broadcast), so the compiler would move
// the whole chain onto the scalar unit (3 SALU per F + readfirstlane
// round-trips).  An empty asm with "v" operands makes them opaque VGPR values
// and keeps the chain on the VALU at 4 instructions per step.
#define HBX_VREG4(w) asm("" : "+v"(w))
#define HBX_STEPW(FN, a, b, c, d, w, s) a = (b) + rotl((a) + (FN(b, c, d)) + (w), s)

// MD5 compression with the per-step words already added to the step
// constants (W_i = M[g(i)] + T_i): 4 VALU per step on the serial chain.
__device__ __forceinline__ void md5_compress_w(uint32_t (&h)[4], const uint32_t* __restrict__ Wl) {
  const u32x4* W4 = reinterpret_cast<const u32x4*>(Wl);
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  u32x4 w;
  w = W4[0];
  HBX_VREG4(w);
  HBX_STEPW(HBX_F, a, b, c, d, w.x, 7); HBX_STEPW(HBX_F, d, a, b, c, w.y, 12);
  HBX_STEPW(HBX_F, c, d, a, b, w.z, 17); HBX_STEPW(HBX_F, b, c, d, a, w.w, 22);
  w = W4[1];
  HBX_VREG4(w);
  HBX_STEPW(HBX_F, a, b, c, d, w.x, 7); HBX_STEPW(HBX_F, d, a, b, c, w.y, 12);
  HBX_STEPW(HBX_F, c, d, a, b, w.z, 17); HBX_STEPW(HBX_F, b, c, d, a, w.w, 22);
  w = W4[2];
  HBX_VREG4(w);
  HBX_STEPW(HBX_F, a, b, c, d, w.x, 7); HBX_STEPW(HBX_F, d, a, b, c, w.y, 12);
  HBX_STEPW(HBX_F, c, d, a, b, w.z, 17); HBX_STEPW(HBX_F, b, c, d, a, w.w, 22);
  w = W4[3];
  HBX_VREG4(w);
  HBX_STEPW(HBX_F, a, b, c, d, w.x, 7); HBX_STEPW(HBX_F, d, a, b, c, w.y, 12);
  HBX_STEPW(HBX_F, c, d, a, b, w.z, 17); HBX_STEPW(HBX_F, b, c, d, a, w.w, 22);
  w = W4[4];
  HBX_VREG4(w);
  HBX_STEPW(HBX_G, a, b, c, d, w.x, 5); HBX_STEPW(HBX_G, d, a, b, c, w.y, 9);
  HBX_STEPW(HBX_G, c, d, a, b, w.z, 14); HBX_STEPW(HBX_G, b, c, d, a, w.w, 20);
  w = W4[5];
  HBX_VREG4(w);
  HBX_STEPW(HBX_G, a, b, c, d, w.x, 5); HBX_STEPW(HBX_G, d, a, b, c, w.y, 9);
  HBX_STEPW(HBX_G, c, d, a, b, w.z, 14); HBX_STEPW(HBX_G, b, c, d, a, w.w, 20);
  w = W4[6];
  HBX_VREG4(w);
  HBX_STEPW(HBX_G, a, b, c, d, w.x, 5); HBX_STEPW(HBX_G, d, a, b, c, w.y, 9);
  HBX_STEPW(HBX_G, c, d, a, b, w.z, 14); HBX_STEPW(HBX_G, b, c, d, a, w.w, 20);
  w = W4[7];
  HBX_VREG4(w);
  HBX_STEPW(HBX_G, a, b, c, d, w.x, 5); HBX_STEPW(HBX_G, d, a, b, c, w.y, 9);
  HBX_STEPW(HBX_G, c, d, a, b, w.z, 14); HBX_STEPW(HBX_G, b, c, d, a, w.w, 20);
  w = W4[8];
  HBX_VREG4(w);
  HBX_STEPW(HBX_H, a, b, c, d, w.x, 4); HBX_STEPW(HBX_H, d, a, b, c, w.y, 11);
  HBX_STEPW(HBX_H, c, d, a, b, w.z, 16); HBX_STEPW(HBX_H, b, c, d, a, w.w, 23);
  w = W4[9];
  HBX_VREG4(w);
  HBX_STEPW(HBX_H, a, b, c, d, w.x, 4); HBX_STEPW(HBX_H, d, a, b, c, w.y, 11);
  HBX_STEPW(HBX_H, c, d, a, b, w.z, 16); HBX_STEPW(HBX_H, b, c, d, a, w.w, 23);
  w = W4[10];
  HBX_VREG4(w);
  HBX_STEPW(HBX_H, a, b, c, d, w.x, 4); HBX_STEPW(HBX_H, d, a, b, c, w.y, 11);
  HBX_STEPW(HBX_H, c, d, a, b, w.z, 16); HBX_STEPW(HBX_H, b, c, d, a, w.w, 23);
  w = W4[11];
  HBX_VREG4(w);
  HBX_STEPW(HBX_H, a, b, c, d, w.x, 4); HBX_STEPW(HBX_H, d, a, b, c, w.y, 11);
  HBX_STEPW(HBX_H, c, d, a, b, w.z, 16); HBX_STEPW(HBX_H, b, c, d, a, w.w, 23);
  w = W4[12];
  HBX_VREG4(w);
  HBX_STEPW(HBX_I, a, b, c, d, w.x, 6); HBX_STEPW(HBX_I, d, a, b, c, w.y, 10);
  HBX_STEPW(HBX_I, c, d, a, b, w.z, 15); HBX_STEPW(HBX_I, b, c, d, a, w.w, 21);
  w = W4[13];
  HBX_VREG4(w);
  HBX_STEPW(HBX_I, a, b, c, d, w.x, 6); HBX_STEPW(HBX_I, d, a, b, c, w.y, 10);
  HBX_STEPW(HBX_I, c, d, a, b, w.z, 15); HBX_STEPW(HBX_I, b, c, d, a, w.w, 21);
  w = W4[14];
  HBX_VREG4(w);
  HBX_STEPW(HBX_I, a, b, c, d, w.x, 6); HBX_STEPW(HBX_I, d, a, b, c, w.y, 10);
  HBX_STEPW(HBX_I, c, d, a, b, w.z, 15); HBX_STEPW(HBX_I, b, c, d, a, w.w, 21);
  w = W4[15];
  HBX_VREG4(w);
  HBX_STEPW(HBX_I, a, b, c, d, w.x, 6); HBX_STEPW(HBX_I, d, a, b, c, w.y, 10);
  HBX_STEPW(HBX_I, c, d, a, b, w.z, 15); HBX_STEPW(HBX_I, b, c, d, a, w.w, 21);
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
}

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

// "Wave mode": one chunk per wave.  The 64 lanes prepare the next block's
// step words in parallel (lane i: W_i = M[g(i)] + T_i, one word each) into an
// LDS double buffer while every lane runs the same serial chain on the
// current block with 4 VALU per step.  Raw data is loaded 4 blocks ahead.
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
  // wave-uniform descriptor from the 4-aligned chunk start; reads past the
  // chunk + slack return 0
  const __amdgpu_buffer_rsrc_t rs =
      make_rsrc_u(reinterpret_cast<const void*>(cp - sh), (sh + len + 64u + 15u) & ~15u);
  const uint32_t T = len + 8u;
  const uint32_t nb = (T + 9u + 63u) >> 6;  // blocks incl. padding
  const uint64_t bits = (uint64_t)T * 8ull;
  // raw dword pair for (block bb, this lane): R[16bb+gi-2], R[16bb+gi-1]
  auto raw_load = [&](uint32_t bb) -> uint2 {
    const uint32_t off = 4u * (16u * bb + gi) - 8u;  // wraps below 0 -> out of range -> 0
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0u, 0));
  };
  auto produce = [&](uint32_t bb, uint2 raw, uint32_t slot) {
    const uint32_t widx = 16u * bb + gi;
    uint32_t m = msg_word(widx, raw.x, raw.y, sh, len);
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
  for (uint32_t b0 = 0; b0 < nb; b0 += 4u) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t b = b0 + (uint32_t)r;
      if (b < nb) {  // wave-uniform
        const int rn = (r + 1) & 3;
        if (b + 1u < nb) produce(b + 1u, ring[rn], (b + 1u) & 1u);
        ring[rn] = raw_load(b + 5u);
        __builtin_amdgcn_sched_barrier(0);
        md5_compress_w(h, wring + (b & 1u) * 64u);
      }
    }
  }
}


// hbx_device.h — device-side building blocks shared by the gfx950 kernels.
//
// Hot path replaced: hashback/store.go:129-166 (rollsum split,
// librsync rollsum == assumption A1) and pkg/core/block.go:96-111 (MD5 block ID).
//
// Closed form of the window digest.  With positions q (index of
// the newest byte of the MIN-byte window, virtual zero bytes before the file)
// and d[q] = x[q] - x[q-MIN]:
//     S1(q) = S1(q-1) + d[q]            (mod 2^16)
//     s2(q) = s2(q-1) + S1(q)           (mod 2^16; the rollout term MIN*(c+31)
//                                        vanishes because MIN = 2^16)
//     S1(-1) = 0, s2(-1) = 2^15         (char offset 31 is odd)
//     D(q)  = s2(q) << 16 | S1(q)       == rollsum Digest() of data[q-MIN+1..q]
// For a run of positions starting at e0 (relative) with A(e) = sum_{i<e} d_i and
// C(e) = sum_{i<e} i*d_i (positions relative to the same origin), the state
// after e positions is
//     S1 = S1_0 + A(e),   s2 = s2_0 + e*S1 - C(e)                      (*)
// so the per-thread start state follows from two PLAIN prefix sums (A, C) —
// no affine composition in the scan.  Everything is computed in u32 and only
// the low 16 bits are used (Z/2^32 -> Z/2^16 is a ring map).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbx {

constexpr uint32_t kMinBlock = 65536u;    // hashback/hashback.go:38 (also the window)
constexpr uint32_t kMaxBlock = 8388608u;  // hashback/hashback.go:37
constexpr uint32_t kSlice = 4096u;        // positions per slice summary
constexpr uint32_t kSliceShift = 12u;

// 64-bit integer min (HIP's min() has no unsigned long overload and would
// silently go through double).
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ---------------------------------------------------------------- DPP ----
// gfx9 DPP controls.
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;

template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
}

// Inclusive wave-wide prefix sum (64 lanes).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += dpp<kRowShr1>(x);
  x += dpp<kRowShr2>(x);
  x += dpp<kRowShr4>(x);
  x += dpp<kRowShr8>(x);
  x += dpp<kRowBcast15, 0xa>(x);
  x += dpp<kRowBcast31, 0xc>(x);
  return x;
}
// Inclusive prefix sum inside each 16-lane row.
__device__ __forceinline__ uint32_t row_incl_sum(uint32_t x) {
  x += dpp<kRowShr1>(x);
  x += dpp<kRowShr2>(x);
  x += dpp<kRowShr4>(x);
  x += dpp<kRowShr8>(x);
  return x;
}
// Wave max; the result is valid in lane 63.
__device__ __forceinline__ uint32_t wave_max_to_lane63(uint32_t x) {
  x = max(x, dpp<kRowShr1>(x));
  x = max(x, dpp<kRowShr2>(x));
  x = max(x, dpp<kRowShr4>(x));
  x = max(x, dpp<kRowShr8>(x));
  x = max(x, dpp<kRowBcast15, 0xa>(x));
  x = max(x, dpp<kRowBcast31, 0xc>(x));
  return x;
}
__device__ __forceinline__ uint32_t readlane(uint32_t x, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, lane);
}
// Wave-uniform max (all lanes get it).
__device__ __forceinline__ uint32_t wave_max_all(uint32_t x) {
  return readlane(wave_max_to_lane63(x), 63);
}
__device__ __forceinline__ int wave_max_all_i(int x) {
  // lanes with -1 are "no value"; bias to unsigned
  return (int)(wave_max_all((uint32_t)(x + 1))) - 1;
}

// ------------------------------------------------------- byte helpers ----
__device__ __forceinline__ uint32_t dot4(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_udot4(a, b, c, false);
}
// Weights (4k, 4k+1, 4k+2, 4k+3) as packed bytes: lane-local position index.
__device__ __forceinline__ constexpr uint32_t jw(int k) {
  return (uint32_t)(4 * k) | ((uint32_t)(4 * k + 1) << 8) | ((uint32_t)(4 * k + 2) << 16) |
         ((uint32_t)(4 * k + 3) << 24);
}

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// Raw buffer descriptor helpers (bounds-checked loads: out of range reads 0).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nbytes,
                                           0x00020000);
}
// Same, with the inputs forced wave-uniform (readfirstlane): the compiler
// cannot always prove a pointer loaded from memory is uniform and would wrap
// every buffer op in a waterfall loop (guide T20).  Callers guarantee the
// values really are uniform.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u(const void* base, uint32_t nbytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)nbytes);
  const void* pu = reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(pu), (short)0, (int)n, 0x00020000);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Load one lane's RUN=64-byte run (16 dwords) through a descriptor.
__device__ __forceinline__ void load_run64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                           uint32_t (&v)[16]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    u32x4 t = bload16(r, voff + 16u * k, soff);
    v[4 * k + 0] = t.x;
    v[4 * k + 1] = t.y;
    v[4 * k + 2] = t.z;
    v[4 * k + 3] = t.w;
  }
}

// Exact (maxD, last position) over positions [lo, hi] of a 64-lane run layout:
// lane l owns slice-relative positions 64l .. 64l+63.  `in` are the run bytes,
// `out` the bytes MIN earlier, (S1, s2) the state before the lane's first
// position.  Sequential, exact, used only by the cut-chain resolver (K2).
__device__ __forceinline__ void run_argmax_exact(const uint32_t (&in)[16], const uint32_t (&out)[16],
                                                 uint32_t S1, uint32_t s2, int base, int lo, int hi,
                                                 uint32_t& bestD, int& bestPos) {
#pragma unroll
  for (int k = 0; k < 16; k++) {
#pragma unroll
    for (int b = 0; b < 4; b++) {
      uint32_t xi = (in[k] >> (8 * b)) & 0xffu;
      uint32_t xo = (out[k] >> (8 * b)) & 0xffu;
      S1 = S1 + xi - xo;
      s2 = s2 + S1;
      uint32_t D = (s2 << 16) | (S1 & 0xffffu);
      int pos = base + 4 * k + b;
      bool ok = (pos >= lo) & (pos <= hi) & (D >= bestD);
      bestD = ok ? D : bestD;
      bestPos = ok ? pos : bestPos;
    }
  }
}

}  // namespace hbx

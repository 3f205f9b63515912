// Aggregate VALU issue rate per SIMD on gfx950, for the integer ops of K1 and
// K3, at 1/2/4/8 waves per SIMD on every CU of the chip.
//
// Round-2's valu_latency.hip stamped only wave 0 of one workgroup, so under the
// SIMD's age-priority arbitration it timed the oldest wave alone.  Here EVERY
// wave stamps its own start and end (s_memtime, shader clock) and its HW_ID /
// XCC_ID, the host groups waves by (XCC, SE, CU, SIMD), and the rate of a SIMD
// is (waves x instructions) / (last end - first start) in its own clock ticks.
// The kernel time from hipEvents and the GRBM_GUI_ACTIVE cycles of a rocprofv3
// --pmc pass over the same binary cross-check the tick count.
//
// Residency is forced by dynamic LDS: one 256-thread workgroup (one wave per
// SIMD) per CU-slot, `k` slots per CU (LDS per workgroup such that exactly k
// fit in 160 KiB), grid = 256 CUs x k, so every SIMD holds k waves at once.
//
// Streams: each wave runs ITER x 16 x NACC independent instructions (NACC
// accumulators, so the dependent latency, 8-9 cycles, is covered even by one
// wave), plus an MD5 mix: 8 independent chains of the 5-op MD5 step
// (v_bitop3 F; v_add a+m; v_add3 +F+K; v_alignbit rotate; v_add +b).
//
//   hipcc --offload-arch=gfx950 -O3 -o valu_issue valu_issue.hip
//   ./valu_issue [csv]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#define REP4(x) x x x x
#define REP16(x) REP4(x) REP4(x) REP4(x) REP4(x)

constexpr int ITER = 256;

struct Rec { uint64_t t0, t1; uint32_t hw, xcc; };

// One "unit" = 8 independent instructions of the op (or 8 MD5 steps, 40 VALU).
template <int OP>
__device__ __forceinline__ void unit(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3,
                                     uint32_t& a4, uint32_t& a5, uint32_t& a6, uint32_t& a7,
                                     uint32_t m, uint32_t k) {
#define ALL8(S) S(a0) S(a1) S(a2) S(a3) S(a4) S(a5) S(a6) S(a7)
  if constexpr (OP == 0) {
#define S(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 1) {
#define S(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 2) {
#define S(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xac" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 3) {
#define S(x) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 4) {
#define S(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 5) {
#define S(x) asm volatile("v_lshl_add_u32 %0, %0, 16, %0" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 6) {
#define S(x) asm volatile("v_add_u16_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:BYTE_1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 7) {
#define S(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 8) {
#define S(x) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 9) {
#define S(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 10) {
#define S(x) asm volatile("v_add_u32_dpp %0, %1, %0 row_shr:1 bound_ctrl:0" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 11) {
#define S(x) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 12) {
#define S(x) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 13) {
#define S(x) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 15) {
#define S(x) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 16) {
#define S(x) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 17) {
#define S(x) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 18) {
#define S(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 19) {
#define S(x) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 20) {
#define S(x) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 21) {
#define S(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 22) {
#define S(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 23) {
#define S(x) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 24) {
#define S(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 25) {
#define S(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 26) {
#define S(x) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 27) {
#define S(x) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 28) {
#define S(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 29) {
#define S(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 30) {
#define S(x) asm volatile("v_add_u16 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 31) {
#define S(x) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "s"(0x5a827999u));
    ALL8(S)
#undef S
  } else if constexpr (OP == 32) {
#define S(x) asm volatile("v_add_u32 %0, 0x5a827999, %0" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 33) {
#define S(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(m) : "vcc");
    ALL8(S)
#undef S
  } else if constexpr (OP == 34) {
#define S(x) asm volatile("v_max_i32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 35) {
#define S(x) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 36) {
#define S(x) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:0" : "=v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 37) {
#define S(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 38) {
#define S(x) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 39) {
#define S(x) asm volatile("v_max_u16 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 40) {
#define S(x) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 41) {
#define S(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(m), "v"(k));
    ALL8(S)
#undef S
  } else if constexpr (OP == 42) {
#define S(x) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
    ALL8(S)
#undef S
  } else if constexpr (OP == 43) {
#define S(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(m));
    ALL8(S)
#undef S
  } else if constexpr (OP == 14) {
    // MD5 step on 8 independent chains: b' = b + rotl(a + m + F(b,c,d) + K, s),
    // chain i keeps (a_i, b_i) with c, d shared (register pressure of the real
    // kernel is not the point; the op mix and the dependence are).
#define S(a, b) { uint32_t f, t;                                               \
      asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=&v"(f) : "v"(b), "v"(m), "v"(k)); \
      asm volatile("v_add_u32 %0, %1, %2" : "=&v"(t) : "v"(a), "v"(m));           \
      asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(t) : "v"(f), "s"(0x5a827999u)); \
      asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(t));                     \
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(a) : "v"(t), "v"(b)); }
    S(a0, a1) S(a2, a3) S(a4, a5) S(a6, a7) S(a1, a0) S(a3, a2) S(a5, a4) S(a7, a6)
#undef S
  }
#undef ALL8
}

template <int OP>
__global__ __launch_bounds__(256) void stream(Rec* rec, uint32_t* sink, uint32_t seed) {
  extern __shared__ uint32_t lds[];  // only forces residency
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 ^ 0x55u, a3 = a0 + 9u;
  uint32_t a4 = a0 * 7u, a5 = a0 ^ 0x1234u, a6 = a0 + 77u, a7 = a0 * 11u;
  uint32_t m = seed * 0x9e3779b9u + threadIdx.x, k = seed ^ 0xabcdefu;
  if (seed == 0xffffffffu) lds[threadIdx.x] = a0;  // keep the allocation
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITER; i++) {
    REP16(unit<OP>(a0, a1, a2, a3, a4, a5, a6, a7, m, k);)
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if ((threadIdx.x & 63) == 0) {
    Rec r;
    r.t0 = t0; r.t1 = t1;
    r.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    r.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r;
  }
}


// ---- the MD5 compression as K3 compiles it (hbx_kernels.hip md5_compress):
// one chain per lane, message in registers, BLOCKS blocks per wave.  XAD = 1:
// the H rounds as v_xor (off the path) + v_xad; 0: one v_bitop3.
#define MF(b, c, d) ((((c) ^ (d)) & (b)) ^ (d))
#define MG(b, c, d) ((((b) ^ (c)) & (d)) ^ (c))
#define MH(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)
#define MI(b, c, d) ((c) ^ ((b) | ~(d)))
#define MSTEP(FN, a, b, c, d, x, t, s) a = (b) + __builtin_rotateleft32((a) + (FN(b, c, d)) + (x) + (t), (s))
__device__ __forceinline__ uint32_t xad_(uint32_t b, uint32_t cd, uint32_t t1) {
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(cd), "v"(t1));
  return r;
}
__device__ __forceinline__ uint32_t xor_(uint32_t c, uint32_t d) {
  uint32_t r;
  asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(c), "v"(d));
  return r;
}
template <int XAD>
__device__ __forceinline__ void mstep_h(uint32_t& a, uint32_t b, uint32_t c, uint32_t d, uint32_t x, uint32_t t,
                                        int s) {
  if constexpr (XAD) a = b + __builtin_rotateleft32(xad_(b, xor_(c, d), a + x + t), s);
  else MSTEP(MH, a, b, c, d, x, t, s);
}
template <int XAD>
__device__ __forceinline__ void md5c(uint32_t (&h)[4], const uint32_t (&m)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  MSTEP(MF, a, b, c, d, m[0], 0xd76aa478u, 7);  MSTEP(MF, d, a, b, c, m[1], 0xe8c7b756u, 12);
  MSTEP(MF, c, d, a, b, m[2], 0x242070dbu, 17); MSTEP(MF, b, c, d, a, m[3], 0xc1bdceeeu, 22);
  MSTEP(MF, a, b, c, d, m[4], 0xf57c0fafu, 7);  MSTEP(MF, d, a, b, c, m[5], 0x4787c62au, 12);
  MSTEP(MF, c, d, a, b, m[6], 0xa8304613u, 17); MSTEP(MF, b, c, d, a, m[7], 0xfd469501u, 22);
  MSTEP(MF, a, b, c, d, m[8], 0x698098d8u, 7);  MSTEP(MF, d, a, b, c, m[9], 0x8b44f7afu, 12);
  MSTEP(MF, c, d, a, b, m[10], 0xffff5bb1u, 17); MSTEP(MF, b, c, d, a, m[11], 0x895cd7beu, 22);
  MSTEP(MF, a, b, c, d, m[12], 0x6b901122u, 7); MSTEP(MF, d, a, b, c, m[13], 0xfd987193u, 12);
  MSTEP(MF, c, d, a, b, m[14], 0xa679438eu, 17); MSTEP(MF, b, c, d, a, m[15], 0x49b40821u, 22);
  MSTEP(MG, a, b, c, d, m[1], 0xf61e2562u, 5);  MSTEP(MG, d, a, b, c, m[6], 0xc040b340u, 9);
  MSTEP(MG, c, d, a, b, m[11], 0x265e5a51u, 14); MSTEP(MG, b, c, d, a, m[0], 0xe9b6c7aau, 20);
  MSTEP(MG, a, b, c, d, m[5], 0xd62f105du, 5);  MSTEP(MG, d, a, b, c, m[10], 0x02441453u, 9);
  MSTEP(MG, c, d, a, b, m[15], 0xd8a1e681u, 14); MSTEP(MG, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
  MSTEP(MG, a, b, c, d, m[9], 0x21e1cde6u, 5);  MSTEP(MG, d, a, b, c, m[14], 0xc33707d6u, 9);
  MSTEP(MG, c, d, a, b, m[3], 0xf4d50d87u, 14); MSTEP(MG, b, c, d, a, m[8], 0x455a14edu, 20);
  MSTEP(MG, a, b, c, d, m[13], 0xa9e3e905u, 5); MSTEP(MG, d, a, b, c, m[2], 0xfcefa3f8u, 9);
  MSTEP(MG, c, d, a, b, m[7], 0x676f02d9u, 14); MSTEP(MG, b, c, d, a, m[12], 0x8d2a4c8au, 20);
  mstep_h<XAD>(a, b, c, d, m[5], 0xfffa3942u, 4);  mstep_h<XAD>(d, a, b, c, m[8], 0x8771f681u, 11);
  mstep_h<XAD>(c, d, a, b, m[11], 0x6d9d6122u, 16); mstep_h<XAD>(b, c, d, a, m[14], 0xfde5380cu, 23);
  mstep_h<XAD>(a, b, c, d, m[1], 0xa4beea44u, 4);  mstep_h<XAD>(d, a, b, c, m[4], 0x4bdecfa9u, 11);
  mstep_h<XAD>(c, d, a, b, m[7], 0xf6bb4b60u, 16); mstep_h<XAD>(b, c, d, a, m[10], 0xbebfbc70u, 23);
  mstep_h<XAD>(a, b, c, d, m[13], 0x289b7ec6u, 4); mstep_h<XAD>(d, a, b, c, m[0], 0xeaa127fau, 11);
  mstep_h<XAD>(c, d, a, b, m[3], 0xd4ef3085u, 16); mstep_h<XAD>(b, c, d, a, m[6], 0x04881d05u, 23);
  mstep_h<XAD>(a, b, c, d, m[9], 0xd9d4d039u, 4);  mstep_h<XAD>(d, a, b, c, m[12], 0xe6db99e5u, 11);
  mstep_h<XAD>(c, d, a, b, m[15], 0x1fa27cf8u, 16); mstep_h<XAD>(b, c, d, a, m[2], 0xc4ac5665u, 23);
  MSTEP(MI, a, b, c, d, m[0], 0xf4292244u, 6);  MSTEP(MI, d, a, b, c, m[7], 0x432aff97u, 10);
  MSTEP(MI, c, d, a, b, m[14], 0xab9423a7u, 15); MSTEP(MI, b, c, d, a, m[5], 0xfc93a039u, 21);
  MSTEP(MI, a, b, c, d, m[12], 0x655b59c3u, 6); MSTEP(MI, d, a, b, c, m[3], 0x8f0ccc92u, 10);
  MSTEP(MI, c, d, a, b, m[10], 0xffeff47du, 15); MSTEP(MI, b, c, d, a, m[1], 0x85845dd1u, 21);
  MSTEP(MI, a, b, c, d, m[8], 0x6fa87e4fu, 6);  MSTEP(MI, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
  MSTEP(MI, c, d, a, b, m[6], 0xa3014314u, 15); MSTEP(MI, b, c, d, a, m[13], 0x4e0811a1u, 21);
  MSTEP(MI, a, b, c, d, m[4], 0xf7537e82u, 6);  MSTEP(MI, d, a, b, c, m[11], 0xbd3af235u, 10);
  MSTEP(MI, c, d, a, b, m[2], 0x2ad7d2bbu, 15); MSTEP(MI, b, c, d, a, m[9], 0xeb86d391u, 21);
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}
constexpr int MD5_BLOCKS = 1024;
template <int XAD>
__global__ __launch_bounds__(256) void md5real(Rec* rec, uint32_t* sink, uint32_t seed) {
  extern __shared__ uint32_t lds[];
  uint32_t m[16];
#pragma unroll
  for (int j = 0; j < 16; j++) m[j] = seed * (j + 1) + threadIdx.x * 0x9e3779b9u;
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  if (seed == 0xffffffffu) lds[threadIdx.x] = m[0];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < MD5_BLOCKS; i++) {
    md5c<XAD>(h, m);
    m[i & 15] ^= h[0];  // a new message each block (keeps the loop honest)
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = h[0] ^ h[1] ^ h[2] ^ h[3];
  if ((threadIdx.x & 63) == 0) {
    Rec r;
    r.t0 = t0; r.t1 = t1;
    r.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    r.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r;
  }
}


// Two independent chains per lane, step-interleaved (ILP inside one wave).
#define MSTEP2(FN, a, b, c, d, x, t, s)                                    \
  { MSTEP(FN, a##0, b##0, c##0, d##0, x##0, t, s); MSTEP(FN, a##1, b##1, c##1, d##1, x##1, t, s); }
__device__ __forceinline__ void md5c2(uint32_t (&h0)[4], const uint32_t (&m0)[16], uint32_t (&h1)[4],
                                      const uint32_t (&m1)[16]) {
  uint32_t a0 = h0[0], b0 = h0[1], c0 = h0[2], d0 = h0[3];
  uint32_t a1 = h1[0], b1 = h1[1], c1 = h1[2], d1 = h1[3];
#define X(j) m##j
  const uint32_t *mm0 = m0, *mm1 = m1;
#define S2(FN, a, b, c, d, j, t, s) { MSTEP(FN, a##0, b##0, c##0, d##0, mm0[j], t, s); MSTEP(FN, a##1, b##1, c##1, d##1, mm1[j], t, s); }
  S2(MF, a, b, c, d, 0, 0xd76aa478u, 7);  S2(MF, d, a, b, c, 1, 0xe8c7b756u, 12);
  S2(MF, c, d, a, b, 2, 0x242070dbu, 17); S2(MF, b, c, d, a, 3, 0xc1bdceeeu, 22);
  S2(MF, a, b, c, d, 4, 0xf57c0fafu, 7);  S2(MF, d, a, b, c, 5, 0x4787c62au, 12);
  S2(MF, c, d, a, b, 6, 0xa8304613u, 17); S2(MF, b, c, d, a, 7, 0xfd469501u, 22);
  S2(MF, a, b, c, d, 8, 0x698098d8u, 7);  S2(MF, d, a, b, c, 9, 0x8b44f7afu, 12);
  S2(MF, c, d, a, b, 10, 0xffff5bb1u, 17); S2(MF, b, c, d, a, 11, 0x895cd7beu, 22);
  S2(MF, a, b, c, d, 12, 0x6b901122u, 7); S2(MF, d, a, b, c, 13, 0xfd987193u, 12);
  S2(MF, c, d, a, b, 14, 0xa679438eu, 17); S2(MF, b, c, d, a, 15, 0x49b40821u, 22);
  S2(MG, a, b, c, d, 1, 0xf61e2562u, 5);  S2(MG, d, a, b, c, 6, 0xc040b340u, 9);
  S2(MG, c, d, a, b, 11, 0x265e5a51u, 14); S2(MG, b, c, d, a, 0, 0xe9b6c7aau, 20);
  S2(MG, a, b, c, d, 5, 0xd62f105du, 5);  S2(MG, d, a, b, c, 10, 0x02441453u, 9);
  S2(MG, c, d, a, b, 15, 0xd8a1e681u, 14); S2(MG, b, c, d, a, 4, 0xe7d3fbc8u, 20);
  S2(MG, a, b, c, d, 9, 0x21e1cde6u, 5);  S2(MG, d, a, b, c, 14, 0xc33707d6u, 9);
  S2(MG, c, d, a, b, 3, 0xf4d50d87u, 14); S2(MG, b, c, d, a, 8, 0x455a14edu, 20);
  S2(MG, a, b, c, d, 13, 0xa9e3e905u, 5); S2(MG, d, a, b, c, 2, 0xfcefa3f8u, 9);
  S2(MG, c, d, a, b, 7, 0x676f02d9u, 14); S2(MG, b, c, d, a, 12, 0x8d2a4c8au, 20);
  S2(MH, a, b, c, d, 5, 0xfffa3942u, 4);  S2(MH, d, a, b, c, 8, 0x8771f681u, 11);
  S2(MH, c, d, a, b, 11, 0x6d9d6122u, 16); S2(MH, b, c, d, a, 14, 0xfde5380cu, 23);
  S2(MH, a, b, c, d, 1, 0xa4beea44u, 4);  S2(MH, d, a, b, c, 4, 0x4bdecfa9u, 11);
  S2(MH, c, d, a, b, 7, 0xf6bb4b60u, 16); S2(MH, b, c, d, a, 10, 0xbebfbc70u, 23);
  S2(MH, a, b, c, d, 13, 0x289b7ec6u, 4); S2(MH, d, a, b, c, 0, 0xeaa127fau, 11);
  S2(MH, c, d, a, b, 3, 0xd4ef3085u, 16); S2(MH, b, c, d, a, 6, 0x04881d05u, 23);
  S2(MH, a, b, c, d, 9, 0xd9d4d039u, 4);  S2(MH, d, a, b, c, 12, 0xe6db99e5u, 11);
  S2(MH, c, d, a, b, 15, 0x1fa27cf8u, 16); S2(MH, b, c, d, a, 2, 0xc4ac5665u, 23);
  S2(MI, a, b, c, d, 0, 0xf4292244u, 6);  S2(MI, d, a, b, c, 7, 0x432aff97u, 10);
  S2(MI, c, d, a, b, 14, 0xab9423a7u, 15); S2(MI, b, c, d, a, 5, 0xfc93a039u, 21);
  S2(MI, a, b, c, d, 12, 0x655b59c3u, 6); S2(MI, d, a, b, c, 3, 0x8f0ccc92u, 10);
  S2(MI, c, d, a, b, 10, 0xffeff47du, 15); S2(MI, b, c, d, a, 1, 0x85845dd1u, 21);
  S2(MI, a, b, c, d, 8, 0x6fa87e4fu, 6);  S2(MI, d, a, b, c, 15, 0xfe2ce6e0u, 10);
  S2(MI, c, d, a, b, 6, 0xa3014314u, 15); S2(MI, b, c, d, a, 13, 0x4e0811a1u, 21);
  S2(MI, a, b, c, d, 4, 0xf7537e82u, 6);  S2(MI, d, a, b, c, 11, 0xbd3af235u, 10);
  S2(MI, c, d, a, b, 2, 0x2ad7d2bbu, 15); S2(MI, b, c, d, a, 9, 0xeb86d391u, 21);
#undef S2
#undef X
  h0[0] += a0; h0[1] += b0; h0[2] += c0; h0[3] += d0;
  h1[0] += a1; h1[1] += b1; h1[2] += c1; h1[3] += d1;
}
template <int DUMMY>
__global__ __launch_bounds__(256) void md5real2(Rec* rec, uint32_t* sink, uint32_t seed) {
  extern __shared__ uint32_t lds[];
  uint32_t m0[16], m1[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    m0[j] = seed * (j + 1) + threadIdx.x * 0x9e3779b9u;
    m1[j] = seed * (j + 7) + threadIdx.x * 0x7f4a7c15u;
  }
  uint32_t h0[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint32_t h1[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  if (seed == 0xffffffffu) lds[threadIdx.x] = m0[0];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < MD5_BLOCKS / 2; i++) {
    md5c2(h0, m0, h1, m1);
    m0[i & 15] ^= h0[0];
    m1[i & 15] ^= h1[0];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = h0[0] ^ h0[1] ^ h1[2] ^ h1[3];
  if ((threadIdx.x & 63) == 0) {
    Rec r;
    r.t0 = t0; r.t1 = t1;
    r.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    r.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r;
  }
}


// Operand-read test: the same ops with every source a DIFFERENT register
// (16 live registers, op i reads r[i+5], r[i+9] (, r[i+13]) and writes r[i]),
// to separate the ALU rate from register-file reads (the single-op streams
// above read the same m/k registers every instruction).
template <int OP>
__global__ __launch_bounds__(256) void distinct(Rec* rec, uint32_t* sink, uint32_t seed) {
  extern __shared__ uint32_t lds[];
  uint32_t r[16];
#pragma unroll
  for (int j = 0; j < 16; j++) r[j] = seed * (j + 3) + threadIdx.x;
  if (seed == 0xffffffffu) lds[threadIdx.x] = r[0];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        uint32_t& d = r[i];
        const uint32_t a = r[(i + 5) & 15], b = r[(i + 9) & 15], c = r[(i + 13) & 15];
        if constexpr (OP == 0) asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
        if constexpr (OP == 1) asm volatile("v_xor_b32_e32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
        if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(d) : "v"(a), "v"(b), "v"(c));
        if constexpr (OP == 3) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
        if constexpr (OP == 4) asm volatile("v_alignbit_b32 %0, %1, %1, 7" : "=v"(d) : "v"(a));
        if constexpr (OP == 5) asm volatile("v_add_u32_e32 %0, 0x5a827999, %1" : "=v"(d) : "v"(a));
        if constexpr (OP == 6) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(d) : "v"(a));
        if constexpr (OP == 7) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(d) : "v"(a));
        if constexpr (OP == 8) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(d) : "v"(a), "v"(b));
        if constexpr (OP == 9) asm volatile("v_add3_u32 %0, %1, %2, 0x10" : "=v"(d) : "v"(a), "v"(b));
        if constexpr (OP == 10) asm volatile("v_alignbit_b32 %0, %1, %2, 7" : "=v"(d) : "v"(a), "v"(b));
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) x ^= r[j];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) {
    Rec rr;
    rr.t0 = t0; rr.t1 = t1;
    rr.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    rr.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = rr;
  }
}


// MD5 steps in inline asm with the constant as a literal in its own
// full-rate v_add (no SGPR constants, no s_mov per step): bitop3 F, add a+x,
// add K, add F, alignbit, add b = four full-rate + one half-rate op.
// IMM: F 0xca (b?c:d), G 0xe4 (d?b:c), H 0x96, I 0x39 (c^(b|~d)).
#define ASTEP(IMM, a, b, c, d, x, K, S)                                                       \
  {                                                                                           \
    uint32_t f_, t_;                                                                          \
    asm volatile("v_bitop3_b32 %1, %3, %4, %5 bitop3:" #IMM "\n\t"                            \
                 "v_add_u32_e32 %2, %0, %6\n\t"                                               \
                 "v_add_u32_e32 %2, " #K ", %2\n\t"                                           \
                 "v_add_u32_e32 %2, %2, %1\n\t"                                               \
                 "v_alignbit_b32 %2, %2, %2, 32-" #S "\n\t"                                   \
                 "v_add_u32_e32 %0, %2, %3"                                                    \
                 : "+v"(a), "=&v"(f_), "=&v"(t_)                                               \
                 : "v"(b), "v"(c), "v"(d), "v"(x));                                            \
  }
#define AROUNDS(ST, m)                                                                                  \
  ST(0xca, a, b, c, d, m[0], 0xd76aa478, 7) ST(0xca, d, a, b, c, m[1], 0xe8c7b756, 12)                  \
  ST(0xca, c, d, a, b, m[2], 0x242070db, 17) ST(0xca, b, c, d, a, m[3], 0xc1bdceee, 22)                 \
  ST(0xca, a, b, c, d, m[4], 0xf57c0faf, 7) ST(0xca, d, a, b, c, m[5], 0x4787c62a, 12)                  \
  ST(0xca, c, d, a, b, m[6], 0xa8304613, 17) ST(0xca, b, c, d, a, m[7], 0xfd469501, 22)                 \
  ST(0xca, a, b, c, d, m[8], 0x698098d8, 7) ST(0xca, d, a, b, c, m[9], 0x8b44f7af, 12)                  \
  ST(0xca, c, d, a, b, m[10], 0xffff5bb1, 17) ST(0xca, b, c, d, a, m[11], 0x895cd7be, 22)               \
  ST(0xca, a, b, c, d, m[12], 0x6b901122, 7) ST(0xca, d, a, b, c, m[13], 0xfd987193, 12)                \
  ST(0xca, c, d, a, b, m[14], 0xa679438e, 17) ST(0xca, b, c, d, a, m[15], 0x49b40821, 22)               \
  ST(0xe4, a, b, c, d, m[1], 0xf61e2562, 5) ST(0xe4, d, a, b, c, m[6], 0xc040b340, 9)                   \
  ST(0xe4, c, d, a, b, m[11], 0x265e5a51, 14) ST(0xe4, b, c, d, a, m[0], 0xe9b6c7aa, 20)                \
  ST(0xe4, a, b, c, d, m[5], 0xd62f105d, 5) ST(0xe4, d, a, b, c, m[10], 0x02441453, 9)                  \
  ST(0xe4, c, d, a, b, m[15], 0xd8a1e681, 14) ST(0xe4, b, c, d, a, m[4], 0xe7d3fbc8, 20)                \
  ST(0xe4, a, b, c, d, m[9], 0x21e1cde6, 5) ST(0xe4, d, a, b, c, m[14], 0xc33707d6, 9)                  \
  ST(0xe4, c, d, a, b, m[3], 0xf4d50d87, 14) ST(0xe4, b, c, d, a, m[8], 0x455a14ed, 20)                 \
  ST(0xe4, a, b, c, d, m[13], 0xa9e3e905, 5) ST(0xe4, d, a, b, c, m[2], 0xfcefa3f8, 9)                  \
  ST(0xe4, c, d, a, b, m[7], 0x676f02d9, 14) ST(0xe4, b, c, d, a, m[12], 0x8d2a4c8a, 20)                \
  ST(0x96, a, b, c, d, m[5], 0xfffa3942, 4) ST(0x96, d, a, b, c, m[8], 0x8771f681, 11)                  \
  ST(0x96, c, d, a, b, m[11], 0x6d9d6122, 16) ST(0x96, b, c, d, a, m[14], 0xfde5380c, 23)               \
  ST(0x96, a, b, c, d, m[1], 0xa4beea44, 4) ST(0x96, d, a, b, c, m[4], 0x4bdecfa9, 11)                  \
  ST(0x96, c, d, a, b, m[7], 0xf6bb4b60, 16) ST(0x96, b, c, d, a, m[10], 0xbebfbc70, 23)                \
  ST(0x96, a, b, c, d, m[13], 0x289b7ec6, 4) ST(0x96, d, a, b, c, m[0], 0xeaa127fa, 11)                 \
  ST(0x96, c, d, a, b, m[3], 0xd4ef3085, 16) ST(0x96, b, c, d, a, m[6], 0x04881d05, 23)                 \
  ST(0x96, a, b, c, d, m[9], 0xd9d4d039, 4) ST(0x96, d, a, b, c, m[12], 0xe6db99e5, 11)                 \
  ST(0x96, c, d, a, b, m[15], 0x1fa27cf8, 16) ST(0x96, b, c, d, a, m[2], 0xc4ac5665, 23)                \
  ST(0x39, a, b, c, d, m[0], 0xf4292244, 6) ST(0x39, d, a, b, c, m[7], 0x432aff97, 10)                  \
  ST(0x39, c, d, a, b, m[14], 0xab9423a7, 15) ST(0x39, b, c, d, a, m[5], 0xfc93a039, 21)                \
  ST(0x39, a, b, c, d, m[12], 0x655b59c3, 6) ST(0x39, d, a, b, c, m[3], 0x8f0ccc92, 10)                 \
  ST(0x39, c, d, a, b, m[10], 0xffeff47d, 15) ST(0x39, b, c, d, a, m[1], 0x85845dd1, 21)                \
  ST(0x39, a, b, c, d, m[8], 0x6fa87e4f, 6) ST(0x39, d, a, b, c, m[15], 0xfe2ce6e0, 10)                 \
  ST(0x39, c, d, a, b, m[6], 0xa3014314, 15) ST(0x39, b, c, d, a, m[13], 0x4e0811a1, 21)                \
  ST(0x39, a, b, c, d, m[4], 0xf7537e82, 6) ST(0x39, d, a, b, c, m[11], 0xbd3af235, 10)                 \
  ST(0x39, c, d, a, b, m[2], 0x2ad7d2bb, 15) ST(0x39, b, c, d, a, m[9], 0xeb86d391, 21)
__device__ __forceinline__ void md5_asm(uint32_t (&h)[4], const uint32_t (&m)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  AROUNDS(ASTEP, m)
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}
// two chains, step-interleaved
#define ASTEP2(IMM, a, b, c, d, x, K, S) ASTEP(IMM, a##0, b##0, c##0, d##0, x##0, K, S) ASTEP(IMM, a##1, b##1, c##1, d##1, x##1, K, S)
#define AROUNDS2(ST)                                                                                   \
  ST(0xca, a, b, c, d, m0[0]*0+mA[0], 0xd76aa478, 7)
__device__ __forceinline__ void md5_asm2(uint32_t (&h0)[4], const uint32_t (&mA)[16], uint32_t (&h1)[4],
                                         const uint32_t (&mB)[16]) {
  uint32_t a0 = h0[0], b0 = h0[1], c0 = h0[2], d0 = h0[3];
  uint32_t a1 = h1[0], b1 = h1[1], c1 = h1[2], d1 = h1[3];
#define ST2(IMM, a, b, c, d, x, K, S) ASTEP(IMM, a##0, b##0, c##0, d##0, mA[x], K, S) ASTEP(IMM, a##1, b##1, c##1, d##1, mB[x], K, S)
#define IDX(j) j
  ST2(0xca, a, b, c, d, 0, 0xd76aa478, 7) ST2(0xca, d, a, b, c, 1, 0xe8c7b756, 12)
  ST2(0xca, c, d, a, b, 2, 0x242070db, 17) ST2(0xca, b, c, d, a, 3, 0xc1bdceee, 22)
  ST2(0xca, a, b, c, d, 4, 0xf57c0faf, 7) ST2(0xca, d, a, b, c, 5, 0x4787c62a, 12)
  ST2(0xca, c, d, a, b, 6, 0xa8304613, 17) ST2(0xca, b, c, d, a, 7, 0xfd469501, 22)
  ST2(0xca, a, b, c, d, 8, 0x698098d8, 7) ST2(0xca, d, a, b, c, 9, 0x8b44f7af, 12)
  ST2(0xca, c, d, a, b, 10, 0xffff5bb1, 17) ST2(0xca, b, c, d, a, 11, 0x895cd7be, 22)
  ST2(0xca, a, b, c, d, 12, 0x6b901122, 7) ST2(0xca, d, a, b, c, 13, 0xfd987193, 12)
  ST2(0xca, c, d, a, b, 14, 0xa679438e, 17) ST2(0xca, b, c, d, a, 15, 0x49b40821, 22)
  ST2(0xe4, a, b, c, d, 1, 0xf61e2562, 5) ST2(0xe4, d, a, b, c, 6, 0xc040b340, 9)
  ST2(0xe4, c, d, a, b, 11, 0x265e5a51, 14) ST2(0xe4, b, c, d, a, 0, 0xe9b6c7aa, 20)
  ST2(0xe4, a, b, c, d, 5, 0xd62f105d, 5) ST2(0xe4, d, a, b, c, 10, 0x02441453, 9)
  ST2(0xe4, c, d, a, b, 15, 0xd8a1e681, 14) ST2(0xe4, b, c, d, a, 4, 0xe7d3fbc8, 20)
  ST2(0xe4, a, b, c, d, 9, 0x21e1cde6, 5) ST2(0xe4, d, a, b, c, 14, 0xc33707d6, 9)
  ST2(0xe4, c, d, a, b, 3, 0xf4d50d87, 14) ST2(0xe4, b, c, d, a, 8, 0x455a14ed, 20)
  ST2(0xe4, a, b, c, d, 13, 0xa9e3e905, 5) ST2(0xe4, d, a, b, c, 2, 0xfcefa3f8, 9)
  ST2(0xe4, c, d, a, b, 7, 0x676f02d9, 14) ST2(0xe4, b, c, d, a, 12, 0x8d2a4c8a, 20)
  ST2(0x96, a, b, c, d, 5, 0xfffa3942, 4) ST2(0x96, d, a, b, c, 8, 0x8771f681, 11)
  ST2(0x96, c, d, a, b, 11, 0x6d9d6122, 16) ST2(0x96, b, c, d, a, 14, 0xfde5380c, 23)
  ST2(0x96, a, b, c, d, 1, 0xa4beea44, 4) ST2(0x96, d, a, b, c, 4, 0x4bdecfa9, 11)
  ST2(0x96, c, d, a, b, 7, 0xf6bb4b60, 16) ST2(0x96, b, c, d, a, 10, 0xbebfbc70, 23)
  ST2(0x96, a, b, c, d, 13, 0x289b7ec6, 4) ST2(0x96, d, a, b, c, 0, 0xeaa127fa, 11)
  ST2(0x96, c, d, a, b, 3, 0xd4ef3085, 16) ST2(0x96, b, c, d, a, 6, 0x04881d05, 23)
  ST2(0x96, a, b, c, d, 9, 0xd9d4d039, 4) ST2(0x96, d, a, b, c, 12, 0xe6db99e5, 11)
  ST2(0x96, c, d, a, b, 15, 0x1fa27cf8, 16) ST2(0x96, b, c, d, a, 2, 0xc4ac5665, 23)
  ST2(0x39, a, b, c, d, 0, 0xf4292244, 6) ST2(0x39, d, a, b, c, 7, 0x432aff97, 10)
  ST2(0x39, c, d, a, b, 14, 0xab9423a7, 15) ST2(0x39, b, c, d, a, 5, 0xfc93a039, 21)
  ST2(0x39, a, b, c, d, 12, 0x655b59c3, 6) ST2(0x39, d, a, b, c, 3, 0x8f0ccc92, 10)
  ST2(0x39, c, d, a, b, 10, 0xffeff47d, 15) ST2(0x39, b, c, d, a, 1, 0x85845dd1, 21)
  ST2(0x39, a, b, c, d, 8, 0x6fa87e4f, 6) ST2(0x39, d, a, b, c, 15, 0xfe2ce6e0, 10)
  ST2(0x39, c, d, a, b, 6, 0xa3014314, 15) ST2(0x39, b, c, d, a, 13, 0x4e0811a1, 21)
  ST2(0x39, a, b, c, d, 4, 0xf7537e82, 6) ST2(0x39, d, a, b, c, 11, 0xbd3af235, 10)
  ST2(0x39, c, d, a, b, 2, 0x2ad7d2bb, 15) ST2(0x39, b, c, d, a, 9, 0xeb86d391, 21)
  h0[0] += a0; h0[1] += b0; h0[2] += c0; h0[3] += d0;
  h1[0] += a1; h1[1] += b1; h1[2] += c1; h1[3] += d1;
}
#include "md5_asm_variants.inc"
template <int CH>
__global__ __launch_bounds__(256) void md5asm(Rec* rec, uint32_t* sink, uint32_t seed) {
  extern __shared__ uint32_t lds[];
  uint32_t m0[16], m1[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    m0[j] = seed * (j + 1) + threadIdx.x * 0x9e3779b9u;
    m1[j] = seed * (j + 7) + threadIdx.x * 0x7f4a7c15u;
  }
  uint32_t h0[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint32_t h1[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  if (seed == 0xffffffffu) lds[threadIdx.x] = m0[0];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < MD5_BLOCKS / (CH >= 20 ? 2 : CH >= 10 ? 1 : CH); i++) {
    if constexpr (CH == 1) {
      md5_asm(h0, m0);
    } else if constexpr (CH >= 10 && CH < 20) {
      if constexpr (CH == 10) md5v_plain(h0, m0);
      if constexpr (CH == 11) md5v_nop(h0, m0);
      if constexpr (CH == 12) md5v_mov(h0, m0);
      if constexpr (CH == 13) md5v_xkfirst(h0, m0);
      if constexpr (CH == 14) md5v_xkfirst_nop(h0, m0);
      if constexpr (CH == 15) md5v_nop_after_r(h0, m0);
      if constexpr (CH == 16) md5v_nop2(h0, m0);
    } else if constexpr (CH >= 20) {
      if constexpr (CH == 20) md5v2_op(h0, m0, h1, m1);
      if constexpr (CH == 21) md5v2_step(h0, m0, h1, m1);
      if constexpr (CH == 22) md5v2_op_nop(h0, m0, h1, m1);
      m1[i & 15] ^= h1[0];
    } else {
      md5_asm2(h0, m0, h1, m1);
      m1[i & 15] ^= h1[0];
    }
    m0[i & 15] ^= h0[0];
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  sink[blockIdx.x * blockDim.x + threadIdx.x] = h0[0] ^ h0[1] ^ h1[2] ^ h1[3];
  if ((threadIdx.x & 63) == 0) {
    Rec r;
    r.t0 = t0; r.t1 = t1;
    r.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    r.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    rec[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = r;
  }
}

typedef void (*KFn)(Rec*, uint32_t*, uint32_t);
struct OpDesc { const char* name; KFn fn; int valu_per_unit; };

#define OPD(n, i, v) { n, stream<i>, v }
static const OpDesc OPS[] = {
    { "distinct v_add_u32 (2 reads)", distinct<0>, 8 },
    { "distinct v_xor_b32 (2 reads)", distinct<1>, 8 },
    { "distinct v_bitop3 (3 reads)", distinct<2>, 8 },
    { "distinct v_add3 (3 reads)", distinct<3>, 8 },
    { "distinct v_alignbit (1 read)", distinct<4>, 8 },
    { "distinct v_add_u32 literal (1 read)", distinct<5>, 8 },
    { "distinct v_mov_b32 (1 read)", distinct<6>, 8 },
    { "distinct v_add_u32 acc (2 reads, dst=src)", distinct<7>, 8 },
    { "distinct v_bitop3 acc (3 reads, dst=src)", distinct<8>, 8 },
    { "distinct v_add3 literal (2 reads)", distinct<9>, 8 },
    { "distinct v_alignbit (2 reads)", distinct<10>, 8 },
    { "md5_real_xad (per STEP)", md5real<1>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5_real_bitop3 (per STEP)", md5real<0>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5_real_2chains (per chain-STEP)", md5real2<0>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5_asm_litK (per STEP)", md5asm<1>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5_asm_litK_2chains (per chain-STEP)", md5asm<2>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v plain (per chain-STEP)", md5asm<10>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v nop (per chain-STEP)", md5asm<11>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v mov (per chain-STEP)", md5asm<12>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v xkfirst (per chain-STEP)", md5asm<13>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v xkfirst_nop (per chain-STEP)", md5asm<14>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v nop_after_r (per chain-STEP)", md5asm<15>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v nop2 (per chain-STEP)", md5asm<16>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v 2ch_op (per chain-STEP)", md5asm<20>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v 2ch_step (per chain-STEP)", md5asm<21>, MD5_BLOCKS * 64 / (ITER * 16) },
    { "md5v 2ch_op_nop (per chain-STEP)", md5asm<22>, MD5_BLOCKS * 64 / (ITER * 16) },
    OPD("v_add_u32", 0, 8),      OPD("v_add3_u32", 1, 8),    OPD("v_bitop3_b32", 2, 8),
    OPD("v_alignbit_b32", 3, 8), OPD("v_xor_b32", 4, 8),     OPD("v_lshl_add_u32", 5, 8),
    OPD("v_add_u16_sdwa", 6, 8), OPD("v_pk_add_u16", 7, 8),  OPD("v_max3_u32", 8, 8),
    OPD("v_fma_f32", 9, 8),      OPD("v_add_u32_dpp", 10, 8), OPD("v_dot4_u32_u8", 11, 8),
    OPD("v_pk_max_u16", 12, 8),  OPD("v_mov_b32", 13, 8),    OPD("md5_step_x8", 14, 40),
    OPD("v_sub_u32", 15, 8),
    OPD("v_lshlrev_b32", 16, 8),
    OPD("v_lshrrev_b32", 17, 8),
    OPD("v_and_b32", 18, 8),
    OPD("v_or_b32", 19, 8),
    OPD("v_max_u32", 20, 8),
    OPD("v_cndmask_b32", 21, 8),
    OPD("v_perm_b32", 22, 8),
    OPD("v_bfe_u32", 23, 8),
    OPD("v_mul_u32_u24", 24, 8),
    OPD("v_mad_u32_u24", 25, 8),
    OPD("v_xad_u32", 26, 8),
    OPD("v_lshl_or_b32", 27, 8),
    OPD("v_and_or_b32", 28, 8),
    OPD("v_or3_b32", 29, 8),
    OPD("v_add_u16_e32", 30, 8),
    OPD("v_add_u32_sgpr", 31, 8),
    OPD("v_add_u32_lit", 32, 8),
    OPD("v_add_co_u32", 33, 8),
    OPD("v_max_i32", 34, 8),
    OPD("v_alignbyte_b32", 35, 8),
    OPD("v_mov_b32_dpp", 36, 8),
    OPD("v_mul_lo_u32", 37, 8),
    OPD("v_sub_u16_e32", 38, 8),
    OPD("v_max_u16_e32", 39, 8),
    OPD("v_lshrrev_b32_v", 40, 8),
    OPD("v_bfi_b32", 41, 8),
    OPD("v_cvt_f32_u32", 42, 8),
    OPD("v_add_f32", 43, 8),
};

int main(int argc, char** argv) {
  const bool csv = argc > 1 && !strcmp(argv[1], "csv");
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int kmax = 8;
  Rec* d_rec; uint32_t* d_sink;
  (void)hipMalloc(&d_rec, sizeof(Rec) * cus * kmax * 4);
  (void)hipMalloc(&d_sink, sizeof(uint32_t) * cus * kmax * 256);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  std::vector<Rec> h(cus * kmax * 4);
  printf("# %s, %d CUs; clock %d kHz (prop)\n", prop.gcnArchName, cus, prop.clockRate);
  printf("# op, waves/SIMD, SIMDs, median cycles per wave-VALU per SIMD (aggregate), p10, p90, "
         "per-wave cycles/VALU (median), kernel ms, implied GHz\n");
  const char* only = argc > 2 ? argv[2] : nullptr;
  for (const OpDesc& op : OPS) {
    if (only && !strstr(op.name, only)) continue;
    for (int k : {1, 2, 4, 8}) {
      const size_t lds = (k == 1) ? 96 * 1024 : (k == 2) ? 64 * 1024 : (k == 4) ? 36 * 1024 : 18 * 1024;
      (void)hipFuncSetAttribute((const void*)op.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      const int grid = cus * k;
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(op.fn, dim3(grid), dim3(256), lds, 0, d_rec, d_sink, 7u + rep);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
        (void)hipEventElapsedTime(&ms, e0, e1);
      }
      const int nw = grid * 4;
      (void)hipMemcpy(h.data(), d_rec, sizeof(Rec) * nw, hipMemcpyDeviceToHost);
      // group by (xcc, se, cu, simd): HW_ID simd_id [5:4], cu_id [11:8], sh_id [12], se_id [15:13]
      std::map<uint32_t, std::vector<const Rec*>> simd;
      for (int w = 0; w < nw; w++) {
        const uint32_t hw = h[w].hw;
        const uint32_t key = (h[w].xcc << 16) | (((hw >> 13) & 7u) << 12) | (((hw >> 12) & 1u) << 11) |
                             (((hw >> 8) & 0xfu) << 4) | ((hw >> 4) & 3u);
        simd[key].push_back(&h[w]);
      }
      const double instr = (double)ITER * 16 * op.valu_per_unit;
      std::vector<double> agg, per;
      int bad = 0;
      for (auto& kv : simd) {
        uint64_t lo = ~0ull, hi = 0;
        for (const Rec* r : kv.second) {
          lo = std::min(lo, r->t0); hi = std::max(hi, r->t1);
          per.push_back((double)(r->t1 - r->t0) / instr);
        }
        if ((int)kv.second.size() != k) bad++;
        agg.push_back((double)(hi - lo) / (instr * kv.second.size()));
      }
      std::sort(agg.begin(), agg.end());
      std::sort(per.begin(), per.end());
      const double med = agg[agg.size() / 2];
      // implied shader clock: the median SIMD's span vs the event time
      const double span_cyc = med * instr * k;
      printf("%s%s, %d, %zu, %.3f, %.3f, %.3f, %.3f, %.4f, %.3f%s\n", csv ? "" : "", op.name, k,
             agg.size(), med, agg[agg.size() / 10], agg[agg.size() * 9 / 10], per[per.size() / 2], ms,
             span_cyc / (ms * 1e6), bad ? " (SIMDs with another wave count present)" : "");
    }
  }
  return 0;
}

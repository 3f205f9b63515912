// hbx_kernels.hip — gfx950 kernels for the rollsum-split + block-ID path.
//
//   K1 hbx_k1_digest_scan  window digest D(q) at every file position, reduced
//                          to one max per 4096-position slice (+ the digest
//                          just before the slice, which IS the rollsum state)
//                          replaces the Rollin/Rollout/Digest loop of
//                          hashback/store.go:141-165 (smtc/rollsum, A1).
//   K2 hbx_k2_cut_chain    the sequential split rule store.go:111-130,166-173:
//                          cut = LAST argmax D over [s+MIN, s+L], L = min(MAX,
//                          N-s), only if L > 2*MIN.  One wave per file.
//   K3 hbx_k3_block_md5    BlockID = MD5(BE32(0) || BE32(len) || chunk)
//                          (pkg/core/block.go:96-111, utils.go:81-84); one lane
//                          per chunk.
//   K4 hbx_k4_content_id   file content id (store.go:187-196): single chunk ->
//                          its id (type 2); else MD5 of the FileChainBlock
//                          (hashback/hashback.go:162-170) with links = ids
//                          (type 3).
// No MFMA anywhere: this is a byte scan plus an integer hash.
#include <type_traits>
#include <utility>

#include "hbx_device.h"

using namespace hbx;

namespace {

// ------------------------------------------------------------------ K1 --
constexpr int kK1Threads = 1024;  // 16 waves; 16 x 4096 B = one MIN window per iteration

// Per-lane in-aggregates of a 64-byte run: half (positions 0..31) and full.
struct RunAgg {
  uint32_t ah, jh, af, jf;
};
__device__ __forceinline__ RunAgg run_aggregates(const uint32_t (&v)[16]) {
  RunAgg r;
  uint32_t a = 0, j = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    a = dot4(v[k], 0x01010101u, a);
    j = dot4(v[k], jw(k), j);
  }
  r.ah = a;
  r.jh = j;
#pragma unroll
  for (int k = 8; k < 16; k++) {
    a = dot4(v[k], 0x01010101u, a);
    j = dot4(v[k], jw(k), j);
  }
  r.af = a;
  r.jf = j;
  return r;
}

// The digest pass over one lane's 64 positions, with the digest kept as ONE
// register per stream, X = s2<<16 | s1:
//   X.lo += in_byte; X.lo -= out_byte   (SDWA: 16-bit result, high half kept)
//   X += X << 16                        (s2 += s1, mod 2^16, low half kept)
// so X IS the digest — 3 VALU per position instead of ~4.25 + hazard nops.
// Two independent streams per lane (positions 0..31 and 32..63).
#define HBX_SDWA_STEP(X, IN, OUT, B)                                                          \
  asm("v_add_u16_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 " \
      "src1_sel:BYTE_" #B "\n\t"                                                              \
      "v_sub_u16_sdwa %0, %0, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 " \
      "src1_sel:BYTE_" #B "\n\t"                                                              \
      "v_lshl_add_u32 %0, %0, 16, %0"                                                        \
      : "+v"(X)                                                                               \
      : "v"(IN), "v"(OUT))

// Four positions (one dword of each stream) plus the running max, in ONE
// asm block: the compiler pads the boundary between two inline-asm blocks
// with an s_nop whenever the second reads a register the first wrote, which
// cost one issue slot per position pair with a block per position.  The two
// streams' ops are interleaved (independent neighbours).
#define HBX_SDWA_POS(B)                                                                    \
  "v_add_u16_sdwa %0, %0, %3 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 "   \
  "src1_sel:BYTE_" #B "\n\t"                                                              \
  "v_add_u16_sdwa %1, %1, %5 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 "   \
  "src1_sel:BYTE_" #B "\n\t"                                                              \
  "v_sub_u16_sdwa %0, %0, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 "   \
  "src1_sel:BYTE_" #B "\n\t"                                                              \
  "v_sub_u16_sdwa %1, %1, %6 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 "   \
  "src1_sel:BYTE_" #B "\n\t"                                                              \
  "v_lshl_add_u32 %0, %0, 16, %0\n\t"                                                     \
  "v_lshl_add_u32 %1, %1, 16, %1\n\t"                                                     \
  "v_max3_u32 %2, %2, %0, %1\n\t"
#define HBX_SDWA_DWORD(XA, XB, M, INA, OUTA, INB, OUTB)                              \
  asm(HBX_SDWA_POS(0) HBX_SDWA_POS(1) HBX_SDWA_POS(2) HBX_SDWA_POS(3)               \
      : "+v"(XA), "+v"(XB), "+v"(M)                                                  \
      : "v"(INA), "v"(OUTA), "v"(INB), "v"(OUTB))

template <bool TAIL>
__device__ __forceinline__ uint32_t digest_pass_sdwa(const uint32_t (&in)[16],
                                                     const uint32_t (&out)[16], uint32_t XA,
                                                     uint32_t XB, uint32_t e_l, uint32_t lim) {
  uint32_t M = 0;
  if (!TAIL) {
#pragma unroll
    for (int k = 0; k < 8; k++) HBX_SDWA_DWORD(XA, XB, M, in[k], out[k], in[8 + k], out[8 + k]);
    return M;
  }
#pragma unroll
  for (int k = 0; k < 8; k++) {
#define HBX_SDWA_PAIR(B)                                            \
    {                                                               \
      HBX_SDWA_STEP(XA, in[k], out[k], B);                          \
      HBX_SDWA_STEP(XB, in[8 + k], out[8 + k], B);                  \
      uint32_t DA = XA, DB = XB;                                    \
      DA = (e_l + 4u * k + B < lim) ? DA : 0u;                      \
      DB = (e_l + 32u + 4u * k + B < lim) ? DB : 0u;                \
      asm("v_max3_u32 %0, %0, %1, %2" : "+v"(M) : "v"(DA), "v"(DB)); \
    }
    HBX_SDWA_PAIR(0) HBX_SDWA_PAIR(1) HBX_SDWA_PAIR(2) HBX_SDWA_PAIR(3)
#undef HBX_SDWA_PAIR
  }
  return M;
}

}  // namespace

// Rollsum state carried between K1 iterations.
struct K1State {
  uint32_t S1c, s2c;  // state before the iteration's first position
  RunAgg pa;          // in-aggregates of the previous run (= this run's "out")
};

// Priming: the state at q0-1 is the digest state of the MIN bytes before q0
// (`halo`, this thread's 64-byte run of it); at q0 == 0 the window is all
// virtual zeros.
__device__ __forceinline__ K1State k1_prime(const uint32_t (&halo)[16], bool at_start,
                                            uint2 (&wtot)[2][16], uint32_t w, uint32_t l,
                                            uint32_t e_l) {
  K1State st;
  if (at_start) {
    st.pa = RunAgg{0u, 0u, 0u, 0u};
    st.S1c = 0u;
    st.s2c = 0x8000u;
    return st;
  }
  st.pa = run_aggregates(halo);
  const uint32_t iA = wave_incl_sum(st.pa.af);
  const uint32_t iC = wave_incl_sum(e_l * st.pa.af + st.pa.jf);
  if (l == 63u) wtot[1][w] = make_uint2(iA, iC);
  __syncthreads();
  const uint2 t = (l < 16u) ? wtot[1][l] : make_uint2(0u, 0u);
  const uint32_t sA = row_incl_sum(t.x), sC = row_incl_sum(t.y);
  st.S1c = readlane(sA, 15);
  st.s2c = 0x8000u - readlane(sC, 15);  // virtual-zero start: s2 = 2^15 - sum k*x_k
  return st;
}

// One 64 KiB iteration: thread (w, l) owns positions e_l .. e_l+63 of it;
// `cur` are their bytes, `out` the bytes MIN earlier.  Returns, wave-uniform,
// the slice's max digest and the digest just before the slice (= state).
__device__ __forceinline__ void k1_iteration(const uint32_t (&cur)[16], const uint32_t (&out)[16],
                                             K1State& st, uint2 (&wtot)[2][16], uint32_t it,
                                             uint32_t w, uint32_t l, uint32_t e_l, uint64_t qs,
                                             uint64_t N, uint32_t& smax, uint32_t& sprev) {
  const RunAgg ca = run_aggregates(cur);
  const uint32_t A_hA = ca.ah - st.pa.ah, J_hA = ca.jh - st.pa.jh;
  const uint32_t A_l = ca.af - st.pa.af, J_l = ca.jf - st.pa.jf;
  const uint32_t C_l = e_l * A_l + J_l;
  const uint32_t iA = wave_incl_sum(A_l);
  const uint32_t iC = wave_incl_sum(C_l);
  if (l == 63u) wtot[it & 1u][w] = make_uint2(iA, iC);
  __syncthreads();
  const uint2 t = (l < 16u) ? wtot[it & 1u][l] : make_uint2(0u, 0u);
  const uint32_t sA = row_incl_sum(t.x), sC = row_incl_sum(t.y);
  const uint32_t WA = w ? readlane(sA, (int)w - 1) : 0u;
  const uint32_t WC = w ? readlane(sC, (int)w - 1) : 0u;
  const uint32_t totA = readlane(sA, 15), totC = readlane(sC, 15);

  // state before the lane's first position (*), then before position 32
  const uint32_t A_pre = WA + (iA - A_l), C_pre = WC + (iC - C_l);
  const uint32_t S1_t = st.S1c + A_pre;
  const uint32_t s2_t = st.s2c + e_l * S1_t - C_pre;
  const uint32_t A_pre2 = A_pre + A_hA, C_pre2 = C_pre + e_l * A_hA + J_hA;
  const uint32_t S1_b = st.S1c + A_pre2;
  const uint32_t s2_b = st.s2c + (e_l + 32u) * S1_b - C_pre2;
  sprev = readlane((s2_t << 16) | (S1_t & 0xffffu), 0);

  uint32_t M;
  const uint32_t XA = (s2_t << 16) | (S1_t & 0xffffu), XB = (s2_b << 16) | (S1_b & 0xffffu);
  if (qs + kMinBlock <= N) {
    M = digest_pass_sdwa<false>(cur, out, XA, XB, e_l, 0u);
  } else {
    M = digest_pass_sdwa<true>(cur, out, XA, XB, e_l, (uint32_t)(N - qs));
  }
  smax = readlane(wave_max_to_lane63(M), 63);

  st.S1c += totA;
  st.s2c -= totC;  // 65536*(...) vanishes mod 2^16
  st.pa = ca;
}

// Slice summary {max, prev} of one wave-iteration: ONE store instruction
// (lanes 0 and 1), always issued — slices past the file end go to the dummy
// slot — so K1-DMA can count its outstanding vector-memory ops exactly.
__device__ __forceinline__ void k1_store_slice(uint2* __restrict__ ssum, uint64_t idx, uint32_t l,
                                               uint32_t smax, uint32_t sprev) {
  if (l < 2u) reinterpret_cast<uint32_t*>(ssum + idx)[l] = l ? sprev : smax;
}

// ---------------------------------------------------------- K1 (LDS-DMA) --
// Same scan; the runs land in LDS by buffer_load ... lds (no VGPR staging),
// two iterations in flight per CU (128 KiB), instead of one in registers.
// Each wave owns 2 private 4 KiB slots (it reads only what it loaded itself,
// so no barrier guards the data); a slot holds 4 pieces of 1 KiB, piece k
// lane l = bytes 16k..16k+15 of lane l's run, so every ds_read_b128 is
// conflict-free.  Vector-memory ops per wave per iteration are exactly 4 DMA
// + 1 slice store, which makes the hand-counted vmcnt waits exact.
typedef uint32_t s32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s32x4 make_srd(const void* base, uint32_t nbytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  s32x4 r;
  r.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  r.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32)) & 0xffffu;
  r.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)nbytes);
  r.w = 0x00020000u;
  return r;
}

// 64 lanes x 16 B from srd[voff + soff] into LDS [lds, lds + 1 KiB).
// HBX_K1_CPOL: cache-policy bits for K1's stream.  Nontemporal by default: K1
// reads each byte once (plus a 64-B halo), and marking its 8.6 GB per launch
// as streaming leaves L2 to K3 beside it (K3 3.61 -> 3.57 ms, default bench
// 2,156/2,165 -> 2,190/2,186 GiB/s; sc1, sc0 sc1: no gain; tools/gpu_ab_lib.sh)
#ifndef HBX_K1_CPOL
#define HBX_K1_CPOL " nt"
#endif
__device__ __forceinline__ void dma16(s32x4 srd, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen" HBX_K1_CPOL " lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds), "s"(soff)
      : "memory");
}

// The four 1 KiB pieces of a wave's iteration in ONE statement (round 6): M0
// set once, the pieces 1 KiB apart through the instruction offset, which the
// LDS-DMA adds to both the memory and the LDS address (LDS = M0 + offset +
// 16 * lane); the per-piece form paid s_nop 4 + 3 s_mov + s_nop 0 per piece,
// 15 issue slots more per iteration (hbx_k1 ISA, -S).
__device__ __forceinline__ void dma16x4(s32x4 srd, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen" HBX_K1_CPOL " lds\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen offset:1024" HBX_K1_CPOL " lds\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen offset:2048" HBX_K1_CPOL " lds\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen offset:3072" HBX_K1_CPOL " lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds), "s"(soff)
      : "memory");
}

constexpr uint32_t kDmaSlot = 4096;  // bytes per wave per iteration

// One workgroup per tile.  Equal tiles finish in whole rounds over the CUs K3
// leaves free: 512 tiles of 16 MiB on 128 free CUs take 4 rounds, on 127 CUs
// 5 — the measured "residency cliff" (K1 3.2 -> 3.9 ms beside K3 as soon as
// 34+ resident batches put K3's chains on a 129th CU).
// tiles[t] = {file, first 64 KiB iteration, iterations, 0}; ssum[slice_base[f]
// + j] = {max digest of slice j, digest before slice j}; ssum[dummy] absorbs
// the writes of slices past a file's end.
extern "C" __global__ __launch_bounds__(kK1Threads, 1) void hbx_k1_digest_scan_dma(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ file_off,
    const uint64_t* __restrict__ file_len, const uint64_t* __restrict__ slice_base,
    const uint4* __restrict__ tiles, uint2* __restrict__ ssum, uint64_t dummy, uint32_t swz) {
  // swz bit 1 (HBX_K1_DMA4=0, A/B): one statement per piece instead of dma16x4;
  // bit 2 (HBX_K1_EARLY=0, A/B): the first DMA after the halo's loads
  const bool dma4 = !(swz & 2u);
  const bool early = !(swz & 4u);
  swz &= 1u;
  __shared__ uint2 wtot[2][16];
  __shared__ __attribute__((aligned(1024))) uint8_t land[kK1Threads / 64][2][kDmaSlot];
  const uint4 td = tiles[blockIdx.x];
  const uint32_t f = td.x;
  const uint64_t N = file_len[f];
  const uint64_t q0 = (uint64_t)td.y * kMinBlock;
  const uint32_t tile_iters = td.z;
  const uint8_t* fb = arena + file_off[f];
  const uint64_t sb = slice_base[f];

  const uint32_t tid = threadIdx.x;
  const uint32_t l = tid & 63u;
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  const uint32_t e_l = w * kSlice + l * 64u;

  const uint64_t rem = N - q0;
  const uint32_t n_it = (uint32_t)umin64(tile_iters, (rem + kMinBlock - 1) / kMinBlock);
  const uint32_t nbytes = (uint32_t)((umin64(rem, (uint64_t)n_it * kMinBlock) + 15ull) & ~15ull);
  const s32x4 srd = make_srd(fb + q0, nbytes);
  const uint32_t lds0 = (uint32_t)(uintptr_t)&land[w][0][0];
  const uint32_t lds1 = (uint32_t)(uintptr_t)&land[w][1][0];
  // Each DMA instruction reads 1 KiB contiguous; with swz 0 lane l takes
  // bytes 16l..16l+15 of the piece, so the LDS slot holds the wave's 4 KiB in
  // file order and the per-lane 64-byte reads take a 4-way bank conflict (a
  // lane reading bytes 16k.. of its own run instead makes the global access
  // strided, round 2).
  // swz (default): each DMA instruction still reads one contiguous 1 KiB, but
  // lane i loads its 16-B unit 4 (i % 16) + i / 16, so LDS holds each 1 KiB
  // transposed (piece p of run r at slot 16 p + r) and the per-lane reads of
  // piece p are 16 contiguous lanes: no bank conflict
  const uint32_t dma_lane = swz ? 64u * (l & 15u) + 16u * (l >> 4) : 16u * l;
  const uint32_t rd_lane = swz ? 64u * (l >> 4) + (l & 15u) : 4u * l;
  const uint32_t rd_step = swz ? 16u : 1u;
  auto issue = [&](uint32_t it, uint32_t lds) {  // 4 DMA ops, always issued
    if (dma4) {
      dma16x4(srd, w * kSlice + dma_lane, it * kMinBlock, lds);
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t voff = w * kSlice + 1024u * k + dma_lane;
      dma16(srd, voff, it * kMinBlock, lds + 1024u * k);
    }
  };
  auto land_read = [&](uint32_t slot, uint32_t (&v)[16]) {
    const u32x4* p = reinterpret_cast<const u32x4*>(&land[w][slot][0]);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const u32x4 t = p[rd_lane + rd_step * k];
      v[4 * k + 0] = t.x;
      v[4 * k + 1] = t.y;
      v[4 * k + 2] = t.z;
      v[4 * k + 3] = t.w;
    }
  };

  // the first two iterations' DMA goes out before the halo's loads, so their
  // latency and the halo's overlap (round 6: one memory round trip per tile
  // fewer; loads complete in order, so the wait for the halo inside k1_prime
  // lands the DMA too)
  if (early) {
    issue(0u, lds0);
    issue(1u, lds1);  // past the tile end: out-of-range reads land zeros, never read
  }
  uint32_t out[16];
#pragma unroll
  for (int k = 0; k < 16; k++) out[k] = 0u;
  if (q0 != 0) load_run64(make_rsrc_u(fb + q0 - kMinBlock, kMinBlock), e_l, 0u, out);
  K1State st = k1_prime(out, q0 == 0, wtot, w, l, e_l);
  // vmcnt(0) through the builtin, which the compiler's wait pass sees (an asm
  // one it does not): with the asm form it added its own vmcnt(0) after the
  // first two iterations' DMA, so every tile's first iteration waited for
  // both (round 6, tests/test_isa.py)
  if (!early) {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt not waited
    issue(0u, lds0);
    issue(1u, lds1);
  }
  // two register sets swap roles each iteration (this run / the run MIN
  // earlier), so no 16-register copy per iteration
  uint32_t run_b[16];
  auto step = [&](uint32_t it, uint32_t (&cur)[16], const uint32_t (&prev)[16]) {
    // outstanding, oldest first: DMA(it), store(it-2), DMA(it+1), store(it-1)
    if (it == 0)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (it == 1)
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    land_read(it & 1u, cur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot consumed before it is refilled
    issue(it + 2u, (it & 1u) ? lds1 : lds0);
    const uint64_t qs = q0 + (uint64_t)it * kMinBlock;
    uint32_t smax, sprev;
    k1_iteration(cur, prev, st, wtot, it, w, l, e_l, qs, N, smax, sprev);
    const bool ok = qs + (uint64_t)w * kSlice < N;
    k1_store_slice(ssum, ok ? sb + ((qs >> kSliceShift) + w) : dummy, l, smax, sprev);
  };
  for (uint32_t it = 0; it < n_it; it += 2u) {
    step(it, run_b, out);
    if (it + 1u < n_it) step(it + 1u, out, run_b);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup exits
}

// ------------------------------------------------------------------ K2 --
namespace {

// Exact (max D, last slice-relative position) over [lo, hi] of slice j.
__device__ void slice_argmax(const uint8_t* fb, uint64_t N, uint64_t j, uint32_t prevD, int lo,
                             int hi, uint32_t& Dm, int& Pm) {
  const uint32_t l = threadIdx.x & 63u;
  const uint64_t sq = j << kSliceShift;
  const uint64_t avail = N - sq;
  const __amdgpu_buffer_rsrc_t ri =
      make_rsrc_u(fb + sq, (uint32_t)((umin64(avail, kSlice) + 15ull) & ~15ull));
  uint32_t in[16], out[16];
  load_run64(ri, l * 64u, 0u, in);
  if (sq >= kMinBlock) {
    const __amdgpu_buffer_rsrc_t ro = make_rsrc_u(fb + sq - kMinBlock, kSlice);
    load_run64(ro, l * 64u, 0u, out);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = 0u;
  }
  uint32_t A = 0, J = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    A = dot4(in[k], 0x01010101u, A) - dot4(out[k], 0x01010101u, 0u);
    J = dot4(in[k], jw(k), J) - dot4(out[k], jw(k), 0u);
  }
  const uint32_t e = l * 64u;
  const uint32_t C = e * A + J;
  const uint32_t xA = wave_incl_sum(A) - A;
  const uint32_t xC = wave_incl_sum(C) - C;
  const uint32_t S1 = (prevD & 0xffffu) + xA;
  const uint32_t s2 = (prevD >> 16) + e * S1 - xC;
  uint32_t bD = 0u;
  int bP = -1;
  run_argmax_exact(in, out, S1, s2, (int)e, lo, hi, bD, bP);
  Dm = wave_max_all(bP >= 0 ? bD : 0u);
  Pm = wave_max_all_i((bP >= 0 && bD == Dm) ? bP : -1);
}

}  // namespace

// interior summaries per lane per round: 32 x 64 lanes covers the 2048
// slices of a MAX-sized candidate range in one round
constexpr int kK2Loads = 32;

extern "C" __global__ __launch_bounds__(64) void hbx_k2_cut_chain(
    const uint8_t* __restrict__ arena, const uint64_t* __restrict__ file_off,
    const uint64_t* __restrict__ file_len, const uint64_t* __restrict__ slice_base,
    const uint2* __restrict__ ssum,
    const uint64_t* __restrict__ cut_base, uint64_t* __restrict__ cut_ends,
    uint32_t* __restrict__ cut_count, uint32_t* __restrict__ zero_word) {
  const uint32_t f = blockIdx.x;
  const uint32_t l = threadIdx.x;
  // K2r's chain counter (which follows on the same stream), zeroed here
  // instead of by a fill dispatch of its own (hbx_engine.hip, lean marks)
  if (zero_word && f == 0u && l == 0u) *zero_word = 0u;
  const uint64_t N = file_len[f];
  const uint8_t* fb = arena + file_off[f];
  const uint64_t sb = slice_base[f];
  const uint64_t cb = cut_base[f];
  uint64_t s = 0;
  uint32_t k = 0;
  while (s < N) {
    const uint64_t L = umin64(kMaxBlock, N - s);  // store.go:116-120
    uint64_t cut;
    if (L <= 2ull * kMinBlock) {  // store.go:129-130: no split candidate
      cut = s + L;
    } else {
      // candidates p in [s+MIN, s+L]  <=>  q = p-1 in [qa, qb]
      const uint64_t qa = s + kMinBlock - 1, qb = s + L - 1;
      const uint64_t ja = qa >> kSliceShift, jb = qb >> kSliceShift;  // jb - ja >= 16
      // interior slices (ja, jb): max + last slice holding it (and the
      // state before it).  A lane's summary loads, and the two edge slices'
      // summaries, are all issued before the first is used: one memory round
      // trip per cut instead of a chain of up to 32.
      const uint2 sA = ssum[sb + ja], sB = ssum[sb + jb];
      uint32_t bv = 0u, by = 0u;
      int64_t bj = -1;
      for (uint64_t j0 = ja + 1; j0 < jb; j0 += 64u * kK2Loads) {
        uint2 v[kK2Loads];
#pragma unroll
        for (int u = 0; u < kK2Loads; u++) {
          const uint64_t j = j0 + 64u * (uint32_t)u + l;
          v[u] = ssum[sb + (j < jb ? j : jb)];  // jb is in the file: a valid slot
        }
#pragma unroll
        for (int u = 0; u < kK2Loads; u++) {
          const uint64_t j = j0 + 64u * (uint32_t)u + l;
          if (j < jb && v[u].x >= bv) {
            bv = v[u].x;
            by = v[u].y;
            bj = (int64_t)j;
          }
        }
      }
      const uint32_t MI = wave_max_all(bj >= 0 ? bv : 0u);
      const uint32_t jrel = wave_max_all((bj >= 0 && bv == MI) ? (uint32_t)(bj - (int64_t)ja) : 0u);
      const uint64_t jI = ja + jrel;
      // the state before slice jI, from the lane that holds it
      const uint64_t hold = __builtin_amdgcn_ballot_w64(bj == (int64_t)jI);
      const uint32_t yI = readlane(by, hold ? (int)__builtin_ctzll(hold) : 0);

      uint32_t Mbest = MI;
      uint64_t qwin = 0;
      int src = 1;  // 0 = first edge slice, 1 = interior, 2 = last edge slice
      // last (partial) slice: wins ties
      if (sB.x >= Mbest) {
        uint32_t D;
        int P;
        slice_argmax(fb, N, jb, sB.y, 0, (int)(qb - (jb << kSliceShift)), D, P);
        if (P >= 0 && D >= Mbest) {
          Mbest = D;
          qwin = (jb << kSliceShift) + (uint64_t)P;
          src = 2;
        }
      }
      // first (partial) slice: must be strictly greater
      if (sA.x > Mbest) {
        uint32_t D;
        int P;
        slice_argmax(fb, N, ja, sA.y, (int)(qa - (ja << kSliceShift)), (int)kSlice - 1, D, P);
        if (P >= 0 && D > Mbest) {
          Mbest = D;
          qwin = (ja << kSliceShift) + (uint64_t)P;
          src = 0;
        }
      }
      if (src == 1) {
        uint32_t D;
        int P;
        slice_argmax(fb, N, jI, yI, 0, (int)kSlice - 1, D, P);
        qwin = (jI << kSliceShift) + (uint64_t)P;
      }
      cut = qwin + 1;
      // defensive: the chain must always advance within [s+MIN, s+L]; a
      // violation can only come from a bug, never stall the wave on it
      if (cut < s + kMinBlock || cut > s + L) cut = s + L;
    }
    if (l == 0) cut_ends[cb + k] = cut;
    k++;
    s = cut;
  }
  if (l == 0) cut_count[f] = k;
}

// -------------------------------------------------------------- MD5 -----
namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
  return __builtin_rotateleft32(x, (uint32_t)s);
}
#define HBX_F(b, c, d) ((((c) ^ (d)) & (b)) ^ (d))
#define HBX_G(b, c, d) ((((b) ^ (c)) & (d)) ^ (c))
#define HBX_I(b, c, d) ((c) ^ ((b) | ~(d)))
#define HBX_STEP(FN, a, b, c, d, x, t, s) a = (b) + rotl((a) + (FN(b, c, d)) + (x) + (t), s)
// A step's critical path is the chain through b (the previous step's result):
// F(b,c,d) -> + (a+x+t) -> rotate -> + b, four dependent VALU ops.  In the H
// rounds F = b ^ (c ^ d), and (b ^ cd) + t1 is ONE v_xad_u32 when c ^ d is
// formed off the path (c and d are older than b): three dependent ops.  Both
// are written as asm: the compiler would otherwise fold b ^ c ^ d back into
// one v_bitop3 and add it with v_add3 (a, x and the constant).
__device__ __forceinline__ uint32_t xor_offpath(uint32_t c, uint32_t d) {
  uint32_t r;
  asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(c), "v"(d));
  return r;
}
__device__ __forceinline__ uint32_t xad(uint32_t b, uint32_t cd, uint32_t t1) {  // (b ^ cd) + t1
  uint32_t r;
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(cd), "v"(t1));
  return r;
}
#define HBX_STEP_H(a, b, c, d, x, t, s)                    \
  {                                                        \
    const uint32_t cd_ = xor_offpath(c, d);                \
    a = (b) + rotl(xad((b), cd_, (a) + (x) + (t)), s);     \
  }

__device__ __forceinline__ void md5_compress(uint32_t (&h)[4], const uint32_t (&m)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  HBX_STEP(HBX_F, a, b, c, d, m[0], 0xd76aa478u, 7);
  HBX_STEP(HBX_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
  HBX_STEP(HBX_F, c, d, a, b, m[2], 0x242070dbu, 17);
  HBX_STEP(HBX_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
  HBX_STEP(HBX_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
  HBX_STEP(HBX_F, d, a, b, c, m[5], 0x4787c62au, 12);
  HBX_STEP(HBX_F, c, d, a, b, m[6], 0xa8304613u, 17);
  HBX_STEP(HBX_F, b, c, d, a, m[7], 0xfd469501u, 22);
  HBX_STEP(HBX_F, a, b, c, d, m[8], 0x698098d8u, 7);
  HBX_STEP(HBX_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
  HBX_STEP(HBX_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
  HBX_STEP(HBX_F, b, c, d, a, m[11], 0x895cd7beu, 22);
  HBX_STEP(HBX_F, a, b, c, d, m[12], 0x6b901122u, 7);
  HBX_STEP(HBX_F, d, a, b, c, m[13], 0xfd987193u, 12);
  HBX_STEP(HBX_F, c, d, a, b, m[14], 0xa679438eu, 17);
  HBX_STEP(HBX_F, b, c, d, a, m[15], 0x49b40821u, 22);
  HBX_STEP(HBX_G, a, b, c, d, m[1], 0xf61e2562u, 5);
  HBX_STEP(HBX_G, d, a, b, c, m[6], 0xc040b340u, 9);
  HBX_STEP(HBX_G, c, d, a, b, m[11], 0x265e5a51u, 14);
  HBX_STEP(HBX_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
  HBX_STEP(HBX_G, a, b, c, d, m[5], 0xd62f105du, 5);
  HBX_STEP(HBX_G, d, a, b, c, m[10], 0x02441453u, 9);
  HBX_STEP(HBX_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
  HBX_STEP(HBX_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
  HBX_STEP(HBX_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
  HBX_STEP(HBX_G, d, a, b, c, m[14], 0xc33707d6u, 9);
  HBX_STEP(HBX_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
  HBX_STEP(HBX_G, b, c, d, a, m[8], 0x455a14edu, 20);
  HBX_STEP(HBX_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
  HBX_STEP(HBX_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
  HBX_STEP(HBX_G, c, d, a, b, m[7], 0x676f02d9u, 14);
  HBX_STEP(HBX_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);
  HBX_STEP_H(a, b, c, d, m[5], 0xfffa3942u, 4);
  HBX_STEP_H(d, a, b, c, m[8], 0x8771f681u, 11);
  HBX_STEP_H(c, d, a, b, m[11], 0x6d9d6122u, 16);
  HBX_STEP_H(b, c, d, a, m[14], 0xfde5380cu, 23);
  HBX_STEP_H(a, b, c, d, m[1], 0xa4beea44u, 4);
  HBX_STEP_H(d, a, b, c, m[4], 0x4bdecfa9u, 11);
  HBX_STEP_H(c, d, a, b, m[7], 0xf6bb4b60u, 16);
  HBX_STEP_H(b, c, d, a, m[10], 0xbebfbc70u, 23);
  HBX_STEP_H(a, b, c, d, m[13], 0x289b7ec6u, 4);
  HBX_STEP_H(d, a, b, c, m[0], 0xeaa127fau, 11);
  HBX_STEP_H(c, d, a, b, m[3], 0xd4ef3085u, 16);
  HBX_STEP_H(b, c, d, a, m[6], 0x04881d05u, 23);
  HBX_STEP_H(a, b, c, d, m[9], 0xd9d4d039u, 4);
  HBX_STEP_H(d, a, b, c, m[12], 0xe6db99e5u, 11);
  HBX_STEP_H(c, d, a, b, m[15], 0x1fa27cf8u, 16);
  HBX_STEP_H(b, c, d, a, m[2], 0xc4ac5665u, 23);
  HBX_STEP(HBX_I, a, b, c, d, m[0], 0xf4292244u, 6);
  HBX_STEP(HBX_I, d, a, b, c, m[7], 0x432aff97u, 10);
  HBX_STEP(HBX_I, c, d, a, b, m[14], 0xab9423a7u, 15);
  HBX_STEP(HBX_I, b, c, d, a, m[5], 0xfc93a039u, 21);
  HBX_STEP(HBX_I, a, b, c, d, m[12], 0x655b59c3u, 6);
  HBX_STEP(HBX_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
  HBX_STEP(HBX_I, c, d, a, b, m[10], 0xffeff47du, 15);
  HBX_STEP(HBX_I, b, c, d, a, m[1], 0x85845dd1u, 21);
  HBX_STEP(HBX_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
  HBX_STEP(HBX_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
  HBX_STEP(HBX_I, c, d, a, b, m[6], 0xa3014314u, 15);
  HBX_STEP(HBX_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
  HBX_STEP(HBX_I, a, b, c, d, m[4], 0xf7537e82u, 6);
  HBX_STEP(HBX_I, d, a, b, c, m[11], 0xbd3af235u, 10);
  HBX_STEP(HBX_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
  HBX_STEP(HBX_I, b, c, d, a, m[9], 0xeb86d391u, 21);
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
}

__device__ __forceinline__ void md5_init(uint32_t (&h)[4]) {
  h[0] = 0x67452301u;
  h[1] = 0xefcdab89u;
  h[2] = 0x98badcfeu;
  h[3] = 0x10325476u;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// One message word of MD5(BE32(0) || BE32(len) || data) given the two raw
// dwords around its data bytes (lo at data byte dpos-sh, hi after it).
__device__ __forceinline__ uint32_t msg_word(uint32_t widx, uint32_t lo, uint32_t hi, uint32_t sh,
                                             uint32_t len) {
  if (widx == 0u) return 0u;
  if (widx == 1u) return bswap32(len);
  const uint32_t dpos = 4u * (widx - 2u);  // data byte index of this word
  const uint32_t raw = alignbyte(hi, lo, sh);
  if (dpos + 4u <= len) return raw;
  if (dpos > len) return 0u;
  const uint32_t nv = len - dpos;  // 0..3 valid bytes, then the 0x80 pad byte
  const uint32_t mask = nv ? ((1u << (8u * nv)) - 1u) : 0u;
  return (raw & mask) | (0x80u << (8u * nv));
}

// Resumable lane-mode MD5 of M = BE32(0) || BE32(len) || data[0..len) (64
// chains per wave, one per lane).  The lane compresses full message blocks
// [b0, b0+cnt) into h and, when `finish`, the 1-2 padded tail blocks after the
// last full block.  `c` is the chunk start.  Reads stay within the chunk +
// 64 bytes (HBX_ARENA_SLACK): every dword holding chunk bytes and never more
// than 63 bytes past the chunk end.
__device__ void md5_tail(const uint8_t* c, uint32_t len, uint32_t (&h)[4], bool finish);

#ifndef HBX_MD5_RING
#define HBX_MD5_RING 8
#endif
// Chunk bytes are read through explicit global (address space 1) pointers.
// A pointer rebuilt from an integer address is generic to the compiler, and a
// generic (flat) load counts against lgkmcnt as well as vmcnt: every wait for
// an LDS read would then also wait for the prefetches still in flight.
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
__device__ __forceinline__ g_u32* gptr32(const void* p) { return (g_u32*)(uintptr_t)p; }
__device__ __forceinline__ g_u32x4* gptr128(uint64_t a) { return (g_u32x4*)a; }

// (Nontemporal loads measured slower: 99 vs 88 ms per batch.)
__device__ __forceinline__ u32x4 md5_load(g_u32x4* p) { return *p; }
template <int RING = HBX_MD5_RING>  // blocks of prefetch (16 VGPRs each)
__device__ void md5_run(const uint8_t* c, uint32_t len, uint32_t (&h)[4], uint32_t b0, uint32_t cnt,
                        bool finish) {
  const uint32_t sh = (uint32_t)reinterpret_cast<uintptr_t>(c) & 3u;
  g_u32* va = gptr32(c - sh);  // raw R[r] = va[r]
  // prefetches clamp to the last block this lane compresses; a lane with
  // nothing to compress reads block b0-1 (always whole data), never block
  // b0 (which may be the tail, up to 72 bytes past the chunk)
  const uint32_t last = cnt ? b0 + cnt - 1u : (b0 ? b0 - 1u : 0u);
  // Block b needs raw dwords R[16b-2 .. 16b+15]: 16 loaded with it (4 x
  // dwordx4 at va+64b, never below the chunk start) plus 2 carried.  Loads
  // run RING blocks ahead through a register ring.  The loop is wave-uniform
  // (bound = the wave's largest cnt; lanes past their own cnt compute and
  // discard) so the compiler keeps exact vmcnt counting and never drains the
  // ring at a divergent join.
  const uint32_t nmax = wave_max_all(cnt);
  const bool any_first = __builtin_amdgcn_ballot_w64(cnt != 0u && b0 == 0u) != 0ull;
  uint32_t c0 = 0u, c1 = 0u;  // R[16b-2], R[16b-1]
  if (b0 != 0u) {
    c0 = va[16u * b0 - 2u];
    c1 = va[16u * b0 - 1u];
  }
  auto blk_src = [&](uint32_t b) { return reinterpret_cast<g_u32x4*>(va + 16u * b); };
  u32x4 ring[RING][4];
#pragma unroll
  for (int r = 0; r < RING; r++) {
    g_u32x4* src = blk_src(min(b0 + (uint32_t)r, last));
#pragma unroll
    for (int i = 0; i < 4; i++) ring[r][i] = md5_load(src + i);
  }
  auto block = [&](int r, uint32_t i, bool refill) {
    uint32_t R[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      R[4 * q + 0] = ring[r][q].x;
      R[4 * q + 1] = ring[r][q].y;
      R[4 * q + 2] = ring[r][q].z;
      R[4 * q + 3] = ring[r][q].w;
    }
    uint32_t m[16];
    // message word j = data word 16b+j-2 = bytes of R[16b+j-2], R[16b+j-1]
    m[0] = alignbyte(c1, c0, sh);
    m[1] = alignbyte(R[0], c1, sh);
#pragma unroll
    for (int j = 2; j < 16; j++) m[j] = alignbyte(R[j - 1], R[j - 2], sh);
    if (i == 0u && any_first) {  // wave-uniform; block 0 carries the framing
      m[0] = b0 == 0u ? 0u : m[0];
      m[1] = b0 == 0u ? bswap32(len) : m[1];
    }
    c0 = R[14];
    c1 = R[15];
    auto do_refill = [&]() {
      g_u32x4* src = blk_src(min(b0 + i + (uint32_t)RING, last));
#pragma unroll
      for (int q = 0; q < 4; q++) ring[r][q] = md5_load(src + q);
    };
    // refill only after the slot's registers are consumed (the aligned
    // words feed v_alignbyte): the load then reuses them and the ring needs
    // no copies at the loop back-edge
    if (refill) do_refill();
    __builtin_amdgcn_sched_barrier(0);  // keep the refill ahead of this block's compression
    uint32_t t[4] = {h[0], h[1], h[2], h[3]};
    md5_compress(t, m);
    const bool live = i < cnt;
#pragma unroll
    for (int q = 0; q < 4; q++) h[q] = live ? t[q] : h[q];
  };
  uint32_t i = 0;
  for (; i + (uint32_t)RING <= nmax; i += (uint32_t)RING) {
#pragma unroll
    for (int r = 0; r < RING; r++) block(r, i + (uint32_t)r, true);
  }
#pragma unroll
  for (int r = 0; r < RING - 1; r++) {
    if (i + (uint32_t)r < nmax) block(r, i + (uint32_t)r, false);
  }
  md5_tail(c, len, h, finish);
}

// The 1-2 padded tail blocks after the last full block (lanes with `finish`).
__device__ void md5_tail(const uint8_t* c, uint32_t len, uint32_t (&h)[4], bool finish) {
  const uint32_t sh = (uint32_t)reinterpret_cast<uintptr_t>(c) & 3u;
  g_u32* va = gptr32(c - sh);
  const uint32_t T = len + 8u;
  const uint32_t nfull = T >> 6;
  // tail: remaining message bytes + 0x80 + zeros + 64-bit bit length
  const uint32_t rem = T - 64u * nfull;  // 0..63
  const uint32_t ntail = finish ? ((rem + 9u > 64u) ? 2u : 1u) : 0u;
  for (uint32_t tb = 0; tb < ntail; tb++) {
    const uint32_t bb = nfull + tb;
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint32_t widx = 16u * bb + (uint32_t)j;
      uint32_t lo = 0u, hi = 0u;
      const uint32_t dpos = 4u * (widx - 2u);
      if (widx >= 2u && dpos < len) {
        lo = va[dpos >> 2];
        hi = va[(dpos >> 2) + 1u];
      }
      m[j] = msg_word(widx, lo, hi, sh, len);
    }
    if (tb + 1 == ntail) {
      const uint64_t bits = (uint64_t)T * 8ull;
      m[14] = (uint32_t)bits;
      m[15] = (uint32_t)(bits >> 32);
    }
    md5_compress(h, m);
  }
}

// One full message block b of a lane's chain through plain per-lane loads
// (the prologue of the cooperative path below: it puts every lane of the
// wave at a block >= 1, where the message words are data words).
__device__ void md5_block_at(const uint8_t* c, uint32_t len, uint32_t (&h)[4], uint32_t b) {
  const uint32_t sh = (uint32_t)reinterpret_cast<uintptr_t>(c) & 3u;
  g_u32* va = gptr32(c - sh);
  const uint32_t base = b ? 16u * b - 2u : 0u;
  uint32_t v[17];
#pragma unroll
  for (int j = 0; j < 17; j++) v[j] = va[base + (uint32_t)j];
  uint32_t m[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t dw = alignbyte(v[j + 1], v[j], sh);                    // b >= 1: word j
    const uint32_t d0 = j >= 2 ? alignbyte(v[j - 1], v[j - 2], sh) : 0u;  // b == 0
    m[j] = b ? dw : (j == 0 ? 0u : j == 1 ? bswap32(len) : d0);
  }
  md5_compress(h, m);
}

// Cooperative streaming for a wave whose 64 lanes all advance exactly R
// blocks, lane j from block b1_j >= 1 of its own chain.  Lane-mode loads put
// 64 chains (64 pages) in every load instruction and the per-CU address
// translation thrashes (89 % UTCL1 misses); here a load
// instruction fetches 16*G contiguous bytes of each of C = 64/G chains, so it
// touches ~C pages.  Each chain's message stream is read from its exact byte
// address S_j = chunk + 64*b1 - 8 (16-B loads at any byte offset; the
// hardware splits them), so the words land aligned and a block needs no
// v_alignbyte.  A stage is G granules (16 B) of every chain = G/4 blocks,
// staged through registers into LDS rows of 16*G + 16 bytes (conflict-free
// ds_read_b128 of a lane's own row), two stages resident (the current one and
// the next); each lane reads its row with 4 aligned ds_read_b128 per block.
//   G = 16: 4-block stages, 272-B rows, 34 KiB per wave (one wave per SIMD).
// (G = 8, 2-block stages for two waves per SIMD, measured 1.9x slower per
// launch at the contract's residency: DESIGN.md §5 K3.)
template <int G>
struct Coop {
  static constexpr uint32_t C = 64u / G;          // chains per load instruction
  static constexpr uint32_t Row = 16u * G + 16u;  // one chain's stage + 16 B pad
  static constexpr uint32_t Half = 64u * Row;     // one stage of the wave's 64 chains
  static constexpr uint32_t WaveLds = 2u * Half;
  static constexpr uint32_t BPS = G / 4u;         // message blocks per stage
};
constexpr uint32_t kCoopWaveLds = Coop<16>::WaveLds;

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src_lane) {
  const int lo = __builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)(uint32_t)v);
  const int hi = __builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Stage registers into LDS half `half` (lane: granule t of the rows C*q+sub).
template <int G>
__device__ __forceinline__ void coop_write(uint8_t* wl, uint32_t wr, uint32_t half, const u32x4 (&Gs)[G]) {
#pragma unroll
  for (int q = 0; q < G; q++)
    *reinterpret_cast<u32x4*>(wl + wr + half * Coop<G>::Half + Coop<G>::C * Coop<G>::Row * (uint32_t)q) = Gs[q];
}

// Loads of stage `st` (granules G*st .. G*st+G-1 of every chain) into Gs.
// Branch-free, so the compiler's vmcnt bookkeeping stays exact through the
// stage loop and a wait covers only the register set it needs: a granule
// past the last needed one (>= ngr) re-reads granule ngr-1, which every
// chain holds.
template <int G>
__device__ __forceinline__ void coop_load(u32x4 (&Gs)[G], const uint64_t (&Q)[G], uint32_t st, uint32_t t,
                                          uint32_t ngr) {
  const uint32_t g = min((uint32_t)G * st + t, ngr - 1u);  // this lane's granule
  const uint64_t off = 16ull * (g - t);                     // Q[q] already holds + 16 t
#pragma unroll
  for (int q = 0; q < G; q++) Gs[q] = md5_load(gptr128(Q[q] + off));
}

// The G/4 blocks of stage s from LDS half `half` (blocks past R skipped).
template <int G>
__device__ __forceinline__ void coop_hash(const uint8_t* wl, uint32_t rd, uint32_t half, uint32_t s, uint32_t R,
                                          uint32_t (&h)[4]) {
  const uint8_t* hb = wl + rd + half * Coop<G>::Half;
#pragma unroll
  for (int u = 0; u < (int)Coop<G>::BPS; u++) {
    const uint32_t blk = Coop<G>::BPS * s + (uint32_t)u;
    if (blk >= R) break;  // wave-uniform
    u32x4 W[4];
#pragma unroll
    for (int i = 0; i < 4; i++) W[i] = *reinterpret_cast<const u32x4*>(hb + 16u * (4u * u + (uint32_t)i));
    const uint32_t m[16] = {W[0].x, W[0].y, W[0].z, W[0].w, W[1].x, W[1].y, W[1].z, W[1].w,
                            W[2].x, W[2].y, W[2].z, W[2].w, W[3].x, W[3].y, W[3].z, W[3].w};
    md5_compress(h, m);
  }
}

// Two register sets of loads in flight: stages s+1 and s+2 while stage s is
// hashed (a third measured no faster).
template <int G>
__device__ void md5_coop(uint8_t* wl, const uint8_t* c, uint32_t (&h)[4], uint32_t b1, uint32_t R) {
  static_assert(G == 16, "stage of 4 blocks");
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t S = reinterpret_cast<uint64_t>(c) + 64ull * b1 - 8ull;  // message block b1
  const uint32_t ngr = 4u * R;                                           // granules of R blocks
  const uint32_t t = lane % (uint32_t)G, sub = lane / (uint32_t)G;
  uint64_t Q[G];  // role q: chain C*q+sub, granule t of each stage
#pragma unroll
  for (int q = 0; q < G; q++) Q[q] = shfl64(S, Coop<G>::C * (uint32_t)q + sub) + 16ull * t;
  const uint32_t wr = sub * Coop<G>::Row + 16u * t;
  const uint32_t rd = lane * Coop<G>::Row;  // this lane's row
  const uint32_t nst = (ngr + (uint32_t)G - 1u) / (uint32_t)G;
  constexpr uint32_t BPS = Coop<G>::BPS;
  // Stages past the last re-read it (coop_load clamps); their writes land in
  // a half never read again.
  u32x4 GA[G], GB[G];
  coop_load<G>(GA, Q, 0u, t, ngr);
  coop_load<G>(GB, Q, 1u, t, ngr);
  coop_write<G>(wl, wr, 0u, GA);
  coop_load<G>(GA, Q, 2u, t, ngr);
  // start of stage s: stage s+1 (in Gn) into the other half, then Gn's
  // registers take the loads of stage s+3
  auto stage = [&](auto half_c, uint32_t s, u32x4(&Gn)[G]) {
    constexpr uint32_t HALF = decltype(half_c)::value;
    coop_write<G>(wl, wr, HALF ^ 1u, Gn);
    coop_load<G>(Gn, Q, min(s + 3u, nst - 1u), t, ngr);
    coop_hash<G>(wl, rd, HALF, s, R, h);
  };
  for (uint32_t s = 0; BPS * s < R; s += 2u) {
    stage(std::integral_constant<uint32_t, 0>{}, s, GB);
    stage(std::integral_constant<uint32_t, 1>{}, s + 1u, GA);  // hashes nothing past block R
  }
}

}  // namespace

// ------------------------------------------------------ MD5 chain table --
// K3 is time-sliced: one launch advances every chain in flight by at most
// `budget` full message blocks (HBX: hbx_set_md5_slice), carrying the MD5
// state in this table between launches.  Chunks of a new batch join the
// table as fresh chains, so several batches pipeline through one stream and
// no batch waits for another's longest chunk (DESIGN.md §4 "K3").
struct alignas(16) Chain {
  uint64_t src;   // device address of the chunk's first byte
  uint32_t len;   // chunk bytes
  uint32_t next;  // full message blocks already compressed; kChainDone once hashed
  uint32_t h[4];  // MD5 state after `next` blocks
  uint64_t out;   // device address of the chunk's 16-byte BlockID
  uint64_t pad;
};
constexpr uint32_t kChainDone = 0xFFFFFFFFu;
constexpr uint32_t kBudgetAll = 0xFFFFFFFFu;

// Full message blocks a launch with `budget` hashes of a chain with `left`
// still to hash.  kSliceRemFirst (round 6, A/B): the chain takes the part
// that does not fill a slice in its FIRST launch ((left - 1) mod budget + 1)
// and a full slice in every later one, instead of full slices first and the
// remainder last.  The launches per chain are the same (ceil(left/budget)),
// so every schedule and completion count holds; what moves is where the
// short counts fall: on the joining batch's chains, which all lie in one
// arena, instead of on chains in their last launch scattered over all of
// them (the launch tail, tools/diag_slow_cu.py).
#ifndef HBX_SLICE_REM_FIRST
#define HBX_SLICE_REM_FIRST 1
#endif
__device__ __forceinline__ uint32_t slice_cnt(uint32_t left, uint32_t budget) {
  if (left <= budget) return left;
  return HBX_SLICE_REM_FIRST ? (left - 1u) % budget + 1u : budget;
}

// ------------------------------------------------------- chain schedule --
// A batch's chains live in the batch's own array for their whole life (K2r
// writes them; K3 updates `next` and the MD5 state in place).  What changes
// from launch to launch is the ORDER in which K3 takes them: a list of
// {chain pointer, full blocks still to hash}, sorted by this launch's block
// count descending in 1024 bins (bin 0 = a full slice), pooled over every
// batch in flight, so the 64 chains of a K3 wave have nearly equal counts and
// the wave advances them together by its minimum (the cooperative path) with
// only a small per-lane remainder.  A chain's progress is deterministic (it
// advances slice_cnt(remaining, budget) blocks per launch), so the planner builds
// the order of launch j from the order of launch j-1 without waiting for K3
// j-1: it runs on the scan stream, beside the hash stream's K3 launches.
struct OrderEntry {
  uint64_t chain;  // Chain* in its batch's array
  uint32_t rem;    // 1 + full message blocks still to hash before this launch (0 = finished)
  uint32_t pad;
};
constexpr uint32_t kPlanBins = 1024u;
__device__ __forceinline__ uint32_t order_bin(uint32_t cnt, uint32_t budget) {
  const uint32_t ref = min(budget, (uint32_t)(kMaxBlock >> 6) + 1u);  // largest possible count
  const uint32_t c = min(cnt, ref);
  return (ref - c) * (kPlanBins - 1u) / ref;
}
// Address-ordered full slices (round 6, the default: 512 bins of 512 MiB
// granules; HBX_PLAN_ADDR / HBX_PLAN_ADDR_SHIFT for A/B): the entries that hash
// a full slice (count == budget: most of a steady-state launch) go to bins
// [0, abins) by their chain's data address in 2^ashift-byte granules (mod
// abins), so a wave's 64 chains, and a CU's four waves (dense placement), read
// a few windows of memory instead of 64 pages anywhere in the resident
// arenas (tools/ubench/hbm_streams: chains within 512 MiB windows 3.41 vs
// 3.10 TB/s spread over 128 GiB, profiles/r06g; K3 3.47-3.49 -> 3.41-3.43 ms,
// launch overhead 1.084-1.089 -> 1.040-1.050, profiles/r06h); the rest by
// descending count in bins [abins, 1024).  Every group of the full-slice
// region still has count == budget, so the K3 walk is unchanged.
__device__ __forceinline__ uint32_t plan_bin(const OrderEntry& o, uint32_t budget, uint32_t abins, uint32_t ashift) {
  const uint32_t cnt = slice_cnt(o.rem - 1u, budget);
  if (!abins) return order_bin(cnt, budget);
  if (cnt == budget) return (uint32_t)((reinterpret_cast<const Chain*>(o.chain)->src >> ashift) % abins);
  const uint32_t ref = min(budget, (uint32_t)(kMaxBlock >> 6) + 1u);
  const uint32_t c = min(cnt, ref);
  return abins + (ref - c) * (kPlanBins - 1u - abins) / ref;
}

// ------------------------------------------------------- K2r new chains --
// One chain per chunk of a new batch, in any order, into the batch's array;
// one order entry per chain into `fresh`; count in cnt[0] (zeroed before).
constexpr uint32_t kPlanLanesPerFile = 16u;  // work items sharing one file's chunks

extern "C" __global__ __launch_bounds__(256) void hbx_k2r_new_chains(
    uint32_t n_files, const uint8_t* __restrict__ arena, const uint64_t* __restrict__ file_off,
    const uint64_t* __restrict__ cut_base, const uint64_t* __restrict__ cut_ends,
    const uint32_t* __restrict__ cut_count, uint32_t* __restrict__ ids, Chain* __restrict__ run,
    OrderEntry* __restrict__ fresh, uint32_t* __restrict__ cnt) {
  const uint32_t w = blockIdx.x * 256u + threadIdx.x;
  if (w >= n_files * kPlanLanesPerFile) return;
  const uint32_t f = w / kPlanLanesPerFile;
  const uint64_t cb = cut_base[f];
  const uint32_t k = cut_count[f];
  const uint64_t base = reinterpret_cast<uint64_t>(arena + file_off[f]);
  for (uint32_t i = w % kPlanLanesPerFile; i < k; i += kPlanLanesPerFile) {
    const uint64_t start = i ? cut_ends[cb + i - 1] : 0ull;
    const uint64_t e = cut_ends[cb + i];
    Chain ch;
    ch.src = base + start;
    ch.len = (uint32_t)(e - start);
    ch.next = 0u;
    ch.h[0] = 0x67452301u;
    ch.h[1] = 0xefcdab89u;
    ch.h[2] = 0x98badcfeu;
    ch.h[3] = 0x10325476u;
    ch.out = reinterpret_cast<uint64_t>(ids + 4u * (cb + i));
    ch.pad = 0ull;
    const uint32_t slot = atomicAdd(cnt, 1u);
    run[slot] = ch;
    OrderEntry o;
    o.chain = reinterpret_cast<uint64_t>(run + slot);
    o.rem = ((ch.len + 8u) >> 6) + 1u;
    o.pad = 0u;
    fresh[slot] = o;
  }
}

// ----------------------------------------------------------- K2c plan --
// The order of one K3 launch: the entries of the previous launch's order
// (`prev`, count *n_prev; their rem less what that launch, with budget
// `bprev`, hashed; the ones it finished dropped) plus the fresh entries of
// the batches joining it (`fs`: up to kMaxFresh lists, list i with count
// *fs.n[i]; a K3 period > 1 joins several batches per launch; either part may
// be absent), binned by this launch's count slice_cnt(rem - 1, budget).  Two launches
// of the same grid over the same
// partition:
//   phase 0: per-workgroup histogram of the bins, added into gh[0, 1024)
//   phase 1: every workgroup scans gh into bin bases, reserves its own range
//            in each bin (one atomic per bin on gh[1024 + bin]) and scatters
//            with LDS atomics; workgroup 0 writes the count to *n_out.
// gh (2 x 1024 u32) is zeroed before phase 0.  Order inside a bin is
// arbitrary; results never depend on it (each chain is independent).
constexpr int kPlanThreads = 1024;
static_assert(kPlanThreads == (int)kPlanBins, "one planner thread per bin");
constexpr uint32_t kPlanGroups = 32u;  // grid of both phases
constexpr int kMaxFresh = 8;           // batches joining one launch (kernel argument by value)
struct FreshSet {
  const OrderEntry* f[kMaxFresh];
  const uint32_t* n[kMaxFresh];
  uint32_t k, pad;
};

extern "C" __global__ __launch_bounds__(kPlanThreads) void hbx_k2c_plan(
    const OrderEntry* __restrict__ prev, const uint32_t* __restrict__ n_prev_p, uint32_t bprev,
    FreshSet fs, uint32_t budget, OrderEntry* __restrict__ out, uint32_t* __restrict__ n_out,
    uint32_t* __restrict__ gh, uint32_t phase) {
  const uint32_t abins = (phase >> 8) & 0xfffu;  // address bins for full slices (plan_bin), 0 = off
  const uint32_t ashift = phase >> 24;            // their granule: 2^ashift bytes
  phase &= 0xffu;
  __shared__ uint32_t hist[kPlanBins], pos[kPlanBins], wsum[kPlanThreads / 64];
  const uint32_t tid = threadIdx.x;
  const uint32_t gt = blockIdx.x * kPlanThreads + tid, gn = gridDim.x * kPlanThreads;
  const uint32_t n_prev = prev ? *n_prev_p : 0u;
  uint32_t fend[kMaxFresh];  // end of fresh list i in the combined list
  uint32_t n_all = n_prev;
#pragma unroll
  for (int i = 0; i < kMaxFresh; i++) {
    n_all += (uint32_t)i < fs.k ? *fs.n[i] : 0u;
    fend[i] = n_all;
  }
  // entry e of the combined list, advanced to this launch (rem 0 = finished)
  auto entry = [&](uint32_t e) {
    OrderEntry o;
    if (e < n_prev) {  // the launch with budget bprev finished it iff its full blocks fit
      o = prev[e];
      o.rem = o.rem - 1u <= bprev ? 0u : o.rem - slice_cnt(o.rem - 1u, bprev);
    } else {
      const OrderEntry* f = fs.f[0];
      uint32_t base = n_prev;
#pragma unroll
      for (int i = 1; i < kMaxFresh; i++)
        if (e >= fend[i - 1]) {
          f = fs.f[i];
          base = fend[i - 1];
        }
      o = f[e - base];
    }
    return o;
  };
  hist[tid] = 0u;
  __syncthreads();
  for (uint32_t e = gt; e < n_all; e += gn) {
    const OrderEntry o = entry(e);
    if (o.rem) atomicAdd(&hist[plan_bin(o, budget, abins, ashift)], 1u);
  }
  __syncthreads();
  if (phase == 0u) {
    if (hist[tid]) atomicAdd(&gh[tid], hist[tid]);
    return;
  }
  {  // exclusive scan of the global bins (one per thread), then this
     // workgroup's range inside each bin
    const uint32_t v = gh[tid];
    const uint32_t inc = wave_incl_sum(v);
    if ((tid & 63u) == 63u) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t before = 0u;
    for (uint32_t wv = 0; wv < (tid >> 6); wv++) before += wsum[wv];
    const uint32_t mine = hist[tid];
    pos[tid] = before + inc - v + (mine ? atomicAdd(&gh[kPlanBins + tid], mine) : 0u);
    if (blockIdx.x == 0 && tid == kPlanThreads - 1) {
      *n_out = before + inc;
      n_out[1] = 0u;  // K3Q's item queue head and tail for this order slot
      n_out[2] = 0u;
    }
  }
  __syncthreads();
  for (uint32_t e = gt; e < n_all; e += gn) {
    const OrderEntry o = entry(e);
    if (o.rem) out[atomicAdd(&pos[plan_bin(o, budget, abins, ashift)], 1u)] = o;
  }
}

// ---------------------------------------------------------- K3 block MD5 --
// Block-ID kernel (lane mode: lane = chain, 64 similar-count chains per wave
// in the planner's order).  Each lane resumes its chain at `next`,
// compresses up to `budget` full blocks and either finishes (tail blocks,
// BlockID stored at `out`, entry marked done) or saves the state for the
// next launch.  grid = one 256-thread workgroup per CU (one wave per SIMD);
// group g runs on wave g % 4 of workgroup g / 4 (dense placement, below).
// The MD5 chain is bound by the issue rate of one wave (DESIGN.md "K3").
// Waves whose 64 chains all hold >= kCoopMinBudget blocks stream them with
// cooperative (page-local) loads.
constexpr uint32_t kCoopMinBudget = 8u;
constexpr int kK3Threads = 256;  // one wave per SIMD
constexpr uint32_t kK3WaveLds = Coop<16>::WaveLds;

// ---------------------------------------------------- K3 producer waves --
// K3P (hbx_k3p_block_md5): each MD5 wave gets a producer wave that issues the
// cooperative global loads of its stages and writes the 272-B LDS rows, so
// the MD5 wave's instruction stream is 4 ds_read_b128 + 320 VALU per block
// (verdict r04 item 1).  The pair hands stages over through two LDS counters,
// cumulative over the launch: flags[0] = stages written, flags[1] = stages
// the MD5 wave is done with.  Stage x lives in LDS half x & 1.  The MD5 wave
// frees the last stage of a group only once the whole group is done (its
// partial rounds and lane remainders stage through the same LDS), so the
// producer writes a group's first two stages only after that.
__device__ __forceinline__ uint32_t k3p_flag(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void k3p_wait_ge(uint32_t* p, uint32_t want) {
  for (;;) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)k3p_flag(p));
    if ((int32_t)(v - want) >= 0) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");  // no LDS access of the stage moves above the wait
}
// The same, counting the polls that found the stage not yet written (the MD5
// wave's waits for its producer; reported by the K3 probe, verdict r05 item 1)
// spin (HBX_K3_SPIN, A/B): re-poll at once instead of after s_sleep 1 (64 cycles)
__device__ __forceinline__ void k3p_wait_ge(uint32_t* p, uint32_t want, uint32_t& polls, bool spin) {
  for (;;) {
    const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)k3p_flag(p));
    if ((int32_t)(v - want) >= 0) break;
    polls++;
    if (!spin) __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void k3p_publish(uint32_t* p, uint32_t v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage's LDS writes (or reads) are done
  if ((threadIdx.x & 63u) == 0u) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The MD5 wave's side of one group: blocks 0..Rr-1 of the cooperative phase
// from the producer's stages S, S+1, ..  Each block's 4 ds_read_b128 are
// issued one block ahead (the next stage's first block once the producer has
// published it), so the LDS latency hides behind a block of VALU; two
// register sets alternate without copies.
//
// The reads and their wait are hand-placed (inline asm): the compiler's own
// wait counting loses track across this loop and waited for the block just
// prefetched (lgkmcnt(3..0) before each block: ~140 of ~1,500 cycles per
// block, tools/ubench/k3_prod floor_cons).  Here one asm issues block b+1's
// 4 reads and then waits lgkmcnt(4): LDS operations of a wave complete in
// order, so "at most the 4 just issued outstanding" means block b's reads have
// landed, whatever older LDS operations (the flag poll, a release) the
// compiler placed in between.  The asm takes block b's registers as in/out
// operands, so no use of them moves above the wait.  No SMEM is issued inside
// the loop (it would count in lgkmcnt out of order).
//
// A stage is freed once its last block is hashed (its reads have landed: the
// block waited for them), except the group's last stage (freed by the caller
// once the group is done).
__device__ __forceinline__ void k3p_consume(uint8_t* wl, uint32_t* flags, uint32_t S, uint32_t Rr, uint32_t (&h)[4],
                                            uint32_t& polls, bool spin) {
  const uint32_t row = (uint32_t)(uintptr_t)(wl + (threadIdx.x & 63u) * Coop<16>::Row);  // LDS address
  auto stage_at = [&](uint32_t k) { return row + ((S + k) & 1u) * Coop<16>::Half; };
  // the 4 reads of a block into N, then wait until only those are outstanding:
  // W (the block read before them) has landed
  auto next_wait = [&](uint32_t a, u32x4(&N)[4], u32x4(&W)[4]) {
    asm volatile(
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:16\n\t"
        "ds_read_b128 %2, %8 offset:32\n\t"
        "ds_read_b128 %3, %8 offset:48\n\t"
        "s_waitcnt lgkmcnt(4)"
        : "=&v"(N[0]), "=&v"(N[1]), "=&v"(N[2]), "=&v"(N[3]), "+v"(W[0]), "+v"(W[1]), "+v"(W[2]), "+v"(W[3])
        : "v"(a)
        : "memory");
  };
  auto hash = [&](const u32x4(&W)[4]) {
    const uint32_t m[16] = {W[0].x, W[0].y, W[0].z, W[0].w, W[1].x, W[1].y, W[1].z, W[1].w,
                            W[2].x, W[2].y, W[2].z, W[2].w, W[3].x, W[3].y, W[3].z, W[3].w};
    md5_compress(h, m);
  };
  const uint32_t nst = (4u * Rr + 15u) / 16u;  // >= 2 (Rr >= kCoopMinBudget - 1)
  u32x4 WA[4], WB[4];
  k3p_wait_ge(&flags[0], S + 1u, polls, spin);
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %4 offset:16\n\t"
      "ds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b128 %3, %4 offset:48"
      : "=&v"(WA[0]), "=&v"(WA[1]), "=&v"(WA[2]), "=&v"(WA[3])
      : "v"(stage_at(0u))
      : "memory");
  // every stage but the last: 4 blocks, each prefetching the next (the 4th
  // the next stage's first, once the producer has published that stage)
  for (uint32_t k = 0; k + 1u < nst; k++) {
    const uint32_t a0 = stage_at(k);
    next_wait(a0 + 64u, WB, WA);
    hash(WA);
    next_wait(a0 + 128u, WA, WB);
    hash(WB);
    next_wait(a0 + 192u, WB, WA);
    hash(WA);
    k3p_wait_ge(&flags[0], S + k + 2u, polls, spin);
    next_wait(stage_at(k + 1u), WA, WB);
    hash(WB);
    asm volatile("" ::: "memory");  // stage k is done (its reads have landed: the blocks waited for them)
    if ((threadIdx.x & 63u) == 0u) __hip_atomic_store(&flags[1], S + k + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // the last stage (1-4 blocks; its first is in WA): no prefetch
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(WA[0]), "+v"(WA[1]), "+v"(WA[2]), "+v"(WA[3]) : : "memory");
  hash(WA);
  const uint8_t* last = wl + (threadIdx.x & 63u) * Coop<16>::Row + ((S + nst - 1u) & 1u) * Coop<16>::Half;
  for (uint32_t u = 1; 4u * (nst - 1u) + u < Rr; u++) {
    u32x4 W[4];
#pragma unroll
    for (int i = 0; i < 4; i++) W[i] = *reinterpret_cast<const u32x4*>(last + 64u * u + 16u * i);
    hash(W);
  }
}

// The group's wave-minimum count and the chain position of this lane, exactly
// as the MD5 wave computes them (both roles walk the same groups).  Only what
// cannot change during the launch is read: the order entry's rem (the
// planner's) and the chain's src and len.  The chain's `next` and state are
// the MD5 wave's to rewrite, and for a group on the lane path it does so
// without waiting for the producer, so a producer that read them after that
// rewrite would see another count (advisor r05: a wrapped kChainDone count
// turned a lane-path group into a cooperative one and put the pair's stage
// counters out of step).
struct K3Group {
  uint64_t src;     // chain bytes
  uint32_t next;    // first full block this launch hashes
  uint32_t cnt, R;
  bool active;
};
__device__ __forceinline__ K3Group k3_group(const OrderEntry* __restrict__ order, uint32_t n_total, uint32_t g,
                                            uint32_t budget) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = 64u * g + lane;
  K3Group G;
  G.active = k < n_total;
  // idle lanes stay alive for the wave-wide loop bound: they run an empty
  // slice over the group's first chain and store nothing
  const OrderEntry o = order[G.active ? k : 64u * g];
  const Chain* chp = reinterpret_cast<const Chain*>(o.chain);
  G.src = chp->src;
  const uint32_t left = o.rem - 1u;  // listed entries have rem >= 1
  G.next = ((chp->len + 8u) >> 6) - left;
  G.cnt = G.active ? slice_cnt(left, budget) : 0u;
  // R = the wave's smallest count: all 64 chains advance R blocks together
  G.R = ~wave_max_all(G.active ? ~G.cnt : 0u);
  return G;
}

// The producer's side of one group: the stages S, S+1, .. of Rr blocks of the
// wave's 64 chains, lane l's chain message stream starting at `src` (16-B
// loads at any byte offset, as md5_coop).  Returns the group's stage count.
// SETS register sets of loads in flight (3 by default: one stage more of
// memory latency hidden than 2, HBX_K3_PSETS=2 for A/B).
template <int SETS = 2>
__device__ __forceinline__ uint32_t k3p_produce(uint8_t* wl, uint32_t* flags, uint32_t S, uint64_t src, uint32_t Rr) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t t = lane % 16u, sub = lane / 16u;
  const uint32_t wr = sub * Coop<16>::Row + 16u * t;
  const uint32_t ngr = 4u * Rr, nst = (ngr + 15u) / 16u;
  uint64_t Q[16];
#pragma unroll
  for (int q = 0; q < 16; q++) Q[q] = shfl64(src, 4u * (uint32_t)q + sub) + 16ull * t;
  u32x4 GA[16], GB[16];
  coop_load<16>(GA, Q, 0u, t, ngr);
  coop_load<16>(GB, Q, min(1u, nst - 1u), t, ngr);
  if (SETS == 3) {
    u32x4 GC[16];
    coop_load<16>(GC, Q, min(2u, nst - 1u), t, ngr);
    // stage x goes to LDS half x & 1 once stage x - 2 is freed (flags[1] >= S + x - 1)
    auto put = [&](uint32_t x, u32x4 (&G)[16]) {
      k3p_wait_ge(&flags[1], x < 2u ? S : S + x - 1u);
      coop_write<16>(wl, wr, (S + x) & 1u, G);
      k3p_publish(&flags[0], S + x + 1u);
      coop_load<16>(G, Q, min(x + 3u, nst - 1u), t, ngr);
    };
    for (uint32_t s = 0; s < nst; s += 3u) {
      put(s, GA);
      if (s + 1u < nst) put(s + 1u, GB);
      if (s + 2u < nst) put(s + 2u, GC);
    }
    return nst;
  }
  for (uint32_t s = 0; s < nst; s += 2u) {
    k3p_wait_ge(&flags[1], s < 2u ? S : S + s - 1u);
    coop_write<16>(wl, wr, (S + s) & 1u, GA);
    k3p_publish(&flags[0], S + s + 1u);
    coop_load<16>(GA, Q, min(s + 2u, nst - 1u), t, ngr);
    if (s + 1u < nst) {
      k3p_wait_ge(&flags[1], s + 1u < 2u ? S : S + s);
      coop_write<16>(wl, wr, (S + s + 1u) & 1u, GB);
      k3p_publish(&flags[0], S + s + 2u);
      coop_load<16>(GB, Q, min(s + 3u, nst - 1u), t, ngr);
    }
  }
  return nst;
}

// ----------------------------------------------------------- K3 items --
// K3Q (hbx_k3q_block_md5): the launch's work is cut into items (g, h), part h
// of P of group g's slice (at most ceil(budget / P) blocks of each chain),
// handed out dynamically: every wave takes the next item from a queue, and
// finishing (g, h) queues (g, h+1).  A chain still advances exactly slice_cnt(rem,
// budget) blocks per launch (the planner's and the engine's schedule are
// unchanged), but its slice may continue on another CU: a CU that runs slow
// (which one varies launch by launch, tools/diag_slow_cu.py) no longer holds
// its groups' whole slices, only the part it is on, and the launch's tail
// shrinks from a slow CU's full slice to about one part.  The queue lives in
// the order slot's control words (octl[1] head, octl[2] tail, zeroed by the
// plan) and q[] (entries tagged with the launch, so no clearing); a part's
// chain states reach the next CU through an agent-scope release (the MD5 wave
// after its stores) and acquire (the wave that takes the next part).
constexpr uint32_t kItemExit = 0xFFFFFFFFu;
constexpr uint32_t kItemSpinTicks = 20000000u;  // 200 ms of s_memrealtime: a lost push, never a normal wait

// One lane's share of a work unit: its chain (or, for a lane with nothing to
// hash in it, a shadow chain with >= R blocks, whose data it reads and
// discards), and the blocks it hashes.
struct K3Lane {
  Chain* chp;
  const uint8_t* src;  // chain bytes the lane reads (its own, or the shadow's)
  uint32_t next;       // first block of `src` the cooperative phase starts from (after the prologue block)
  uint32_t len, b0, cnt;
  bool finish, live;   // finish: tail blocks + id; live: its chain state is written back
  uint32_t h[4];
};
template <bool ITEMS>
__device__ __forceinline__ K3Lane k3_lane(const OrderEntry* __restrict__ order, uint32_t n_total, uint32_t g,
                                          uint32_t part, uint32_t budget, uint32_t per_part) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = 64u * g + lane;
  const bool active = k < n_total;
  K3Lane L;
  if constexpr (!ITEMS) {
    // idle lanes stay alive for the wave-wide loop bound: they run an empty
    // slice over the group's first chain and store nothing
    // counts from the order entry, as the producer wave computes them
    // (k3_group): the chain's own `next` agrees with it by the planner's
    // invariant (rem = 1 + full blocks left), but only rem is read by both
    const OrderEntry o = order[active ? k : 64u * g];
    L.chp = reinterpret_cast<Chain*>(o.chain);
    const Chain ch = *L.chp;
    const uint32_t left = o.rem - 1u;
    L.next = ((ch.len + 8u) >> 6) - left;
    L.len = active ? ch.len : 0u;
    L.b0 = active ? L.next : 0u;
    L.cnt = active ? slice_cnt(left, budget) : 0u;
    L.finish = active && left <= budget;
    L.live = active;
    L.src = reinterpret_cast<const uint8_t*>(ch.src);
    L.h[0] = ch.h[0];
    L.h[1] = ch.h[1];
    L.h[2] = ch.h[2];
    L.h[3] = ch.h[3];
  } else {
    const OrderEntry o = order[active ? k : 64u * g];
    L.chp = reinterpret_cast<Chain*>(o.chain);
    Chain ch = *L.chp;
    // the fields a previous part (maybe on another CU or XCD) stored: loaded
    // past the non-coherent caches (agent-scope atomics), no cache-wide fence
    ch.next = __hip_atomic_load(&L.chp->next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < 4; i++) ch.h[i] = __hip_atomic_load(&L.chp->h[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t nfull = (ch.len + 8u) >> 6;
    // this launch's slice of the chain: the planner's rem (1 + blocks left
    // before the launch) and the budget; part `part` of it
    const uint32_t total = slice_cnt(o.rem - 1u, budget);
    const uint32_t start = nfull - (o.rem - 1u);
    const uint64_t lo64 = (uint64_t)part * per_part;
    const uint32_t lo = lo64 < total ? (uint32_t)lo64 : total;
    const uint32_t hi = (uint64_t)lo + per_part < total ? lo + per_part : total;
    const uint32_t last = total ? (total - 1u) / per_part : 0u;  // the part that finishes it
    L.live = active && part <= last && ch.next != kChainDone;
    L.len = L.live ? ch.len : 0u;
    L.b0 = L.live ? ch.next : 0u;  // == start + lo
    L.cnt = L.live ? hi - lo : 0u;
    L.finish = L.live && part == last && start + total == nfull;
    (void)start;
    L.src = reinterpret_cast<const uint8_t*>(ch.src);
    L.next = ch.next;
    L.h[0] = ch.h[0];
    L.h[1] = ch.h[1];
    L.h[2] = ch.h[2];
    L.h[3] = ch.h[3];
    // lanes with nothing to hash here shadow the lane with the most blocks
    // (a lane that only finishes -- its tail blocks, no full block -- keeps
    // its own chain, and k3_wave_R then sends the wave down the lane path)
    const uint32_t mx = wave_max_all(L.cnt);
    if (mx) {
      const int Ls = __builtin_ctzll(__builtin_amdgcn_ballot_w64(L.cnt == mx));
      const uint64_t sa = reinterpret_cast<uint64_t>(L.src);
      const uint64_t ss = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(sa >> 32), Ls) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sa, Ls);
      const uint32_t ns = (uint32_t)__builtin_amdgcn_readlane((int)L.next, Ls);
      if (L.cnt == 0u && !L.finish) {
        L.src = reinterpret_cast<const uint8_t*>(ss);
        L.next = ns;
      }
    }
  }
  return L;
}
// R = the wave's smallest count over the lanes that hash: all 64 chains
// advance R blocks together through page-local cooperative loads (the others
// shadow a chain with >= R blocks), then each lane its own remainder
template <bool ITEMS>
__device__ __forceinline__ uint32_t k3_wave_R(const K3Lane& L) {
  if constexpr (!ITEMS) return ~wave_max_all(L.live ? ~L.cnt : 0u);
  // items: over the lanes that hash here (a lane that only finishes counts
  // with 0: the lane path); none at all -> 0
  const uint32_t m = wave_max_all((L.cnt || L.finish) ? ~L.cnt : 0u);
  return m ? ~m : 0u;
}

// The MD5 wave takes the launch's next item (lane 0, broadcast); items
// [0, G) are the groups' first parts, later ones come from q as parts finish.
__device__ __forceinline__ uint32_t k3q_pop(uint32_t* __restrict__ qc, const uint64_t* __restrict__ q, uint32_t G,
                                            uint32_t total, uint32_t tag, uint32_t* __restrict__ err) {
  uint32_t item = kItemExit;
  if ((threadIdx.x & 63u) == 0u) {
    const uint32_t sl = __hip_atomic_fetch_add(&qc[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sl < G) {
      item = sl;
    } else if (sl < total) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        const uint64_t v = __hip_atomic_load(&q[sl - G], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(v >> 32) == tag) {
          item = (uint32_t)v;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)kItemSpinTicks) {  // never expected: stop, report
          if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  }
  return (uint32_t)__builtin_amdgcn_readlane((int)item, 0);
}
// After a part's chain states are stored (agent-scope atomic stores, drained
// here): queue the next part.  (Agent-scope fences instead write back and
// invalidate the XCD's whole L2 per part: K3 3.45 -> 3.56 ms at 4 parts,
// 3.79 at 8, profiles/r05h.)
__device__ __forceinline__ void k3q_push(uint32_t* __restrict__ qc, uint64_t* __restrict__ q, uint32_t tag,
                                         uint32_t item) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (flat stores count in both)
  if ((threadIdx.x & 63u) == 0u) {
    const uint32_t t = __hip_atomic_fetch_add(&qc[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&q[t], ((uint64_t)tag << 32) | item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The producer wave of pair `flags`: the same groups as its MD5 wave; for a
// group on the cooperative path (R >= kCoopMinBudget), the stages of blocks
// next+1 .. next+R-1 of its 64 chains, SETS register sets in flight.
template <int SETS>
__device__ void k3p_producer(uint8_t* wl, uint32_t* flags, const OrderEntry* __restrict__ order,
                             const uint32_t* __restrict__ n_order, uint32_t budget, uint32_t g0, uint32_t nwaves) {
  const uint32_t n_total = *n_order;
  const uint32_t groups = (n_total + 63u) / 64u;
  uint32_t S = 0;  // stages of this launch so far
  for (uint32_t g = g0; g < groups; g += nwaves) {
    const K3Group G = k3_group(order, n_total, g, budget);
    if (G.R < kCoopMinBudget) continue;  // wave-uniform: the MD5 wave takes the lane path
    S += k3p_produce<SETS>(wl, flags, S, G.src + 64ull * (G.next + 1u) - 8ull, G.R - 1u);  // from block next+1
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (clamped re-reads of the last stage)
}
// K3Q's producer: the items its MD5 wave announces (flags[2] = item, flags[3]
// = items announced), until kItemExit.
__device__ void k3q_producer(uint8_t* wl, uint32_t* flags, const OrderEntry* __restrict__ order,
                             const uint32_t* __restrict__ n_order, uint32_t budget, uint32_t parts,
                             uint32_t per_part) {
  const uint32_t n_total = *n_order;
  const uint32_t G = (n_total + 63u) / 64u;
  uint32_t S = 0;
  for (uint32_t seq = 1;; seq++) {
    k3p_wait_ge(&flags[3], seq);
    const uint32_t item = (uint32_t)__builtin_amdgcn_readfirstlane((int)k3p_flag(&flags[2]));
    if (item == kItemExit) break;
    const K3Lane L = k3_lane<true>(order, n_total, item % G, item / G, budget, per_part);
    const uint32_t R = k3_wave_R<true>(L);
    if (R < kCoopMinBudget) continue;  // the MD5 wave takes the lane path
    S += k3p_produce(wl, flags, S, reinterpret_cast<uint64_t>(L.src) + 64ull * (L.next + 1u) - 8ull, R - 1u);
  }
  (void)parts;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One wave's share of a K3 launch (VGPR + AGPR, no scratch).  `wl` = this
// wave's LDS.  PROD: a producer wave feeds the cooperative stages (K3P,
// `flags` = the pair's counters); else the wave loads and stages them itself.
// ITEMS (K3Q, with PROD): the work comes as items from the launch's queue
// (`qc`, `q`, `tag`; `parts` per group) instead of groups g0, g0 + nwaves, ..
struct K3Queue {
  uint32_t* qc;
  uint64_t* q;
  uint32_t tag, parts;
  uint32_t* err;
};
template <bool PROD, bool ITEMS = false>
__device__ __forceinline__ void k3_body(
    uint8_t* wl, const OrderEntry* __restrict__ order, const uint32_t* __restrict__ n_order, uint32_t budget,
    uint32_t* __restrict__ started, uint32_t t_first, uint32_t t_last, uint64_t* __restrict__ tslot,
    uint64_t* __restrict__ probe, uint32_t* flags = nullptr, K3Queue Q = K3Queue{}, bool spin = false) {
  static_assert(PROD || !ITEMS, "items need the producer waves");
  // the MD5 chains are issue-bound: win the SIMD's issue arbitration against
  // co-resident waves of other kernels
  __builtin_amdgcn_s_setprio(3);
  // dispatch counter for the next batch's K1 gate (hbx_k1_gate): one vector
  // atomic per workgroup as it starts.  Its ticket also times the launch: the
  // workgroup that draws t_first (the launch's first) stamps the start, the
  // wave that draws t_last on started[1] (the launch's last) the end, into
  // tslot (pinned host memory; hbx_engine harvest_k3)
  if (started && threadIdx.x == 0) {
    const uint32_t tk = __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (tslot && tk == t_first) tslot[0] = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t n_total = *n_order;
  const uint32_t groups = (n_total + 63u) / 64u;
  const uint32_t nwaves = gridDim.x * (kK3Threads / 64);
  // dense: group g on wave g % 4 of workgroup g / 4, so the busy waves fill
  // the fewest CUs and whole CUs stay free for the scan stream's K1/K2
  // (spreading one busy wave per CU first measured 1,255 vs 1,510 GiB/s).  The groups are in descending block count, so a CU's four
  // waves end together and the CUs of the short ones free up early for K1.
  // (Dealing the groups round-robin over ceil(groups / 4) workgroups rounded
  // to a multiple of the 8 XCDs, to even out K3's CUs per XCD, mixed long and
  // short waves on every CU: K3 3.52 -> 3.41 ms but K1 3.25 -> 3.54 ms beside
  // it, 2,235 -> 2,091 GiB/s at 33 resident batches.)  K3Q keeps the same
  // waves busy (the first `groups` of them) and hands them items instead.
  const uint32_t g0 = blockIdx.x * (kK3Threads / 64) + wave;
  const uint32_t per_part = ITEMS ? (budget == kBudgetAll ? kBudgetAll : (budget + Q.parts - 1u) / Q.parts) : 0u;
  // diagnostics (hbx_set_k3_probe): per wave its start, the end of its first
  // group's start-up (loads + prologue), its end, R and the largest count
  const uint64_t pt0 = probe ? __builtin_amdgcn_s_memrealtime() : 0ull;
  uint64_t pt1 = 0ull, pc1 = 0ull, pc2 = 0ull, pt2 = 0ull;  // + the first group's cooperative phase, in cycles
  uint32_t pR = 0u, pmax = 0u;
  uint32_t S = 0;  // PROD: stages of this launch so far (the producer counts the same)
  uint32_t seq = 0;  // ITEMS: items announced to the producer
  uint32_t polls = 0;  // PROD: polls that found the producer's stage not yet written
  bool first = true;
  for (uint32_t g = g0;; g += nwaves) {
    uint32_t part = 0u, item = 0u;
    if constexpr (ITEMS) {
      item = g0 < groups ? k3q_pop(Q.qc, Q.q, groups, groups * Q.parts, Q.tag, Q.err) : kItemExit;
      if ((threadIdx.x & 63u) == 0u) {  // announce it to the producer (kItemExit: it stops too)
        __hip_atomic_store(&flags[2], item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      k3p_publish(&flags[3], ++seq);
      if (item == kItemExit) break;
      g = item % groups;
      part = item / groups;
    } else {
      if (g >= groups) break;
    }
    K3Lane L = k3_lane<ITEMS>(order, n_total, g, part, budget, per_part);
    uint32_t(&h)[4] = L.h;
    const uint8_t* src = L.src;
    const uint32_t len = L.len, b0 = L.b0, cnt = L.cnt;
    const bool finish = L.finish;
    const uint32_t R = k3_wave_R<ITEMS>(L);
    if (R >= kCoopMinBudget) {  // wave-uniform
      md5_block_at(src, len, h, L.next);  // every lane now at a block >= 1
      if (probe && first) {
        pt1 = __builtin_amdgcn_s_memrealtime();
        pc1 = __builtin_amdgcn_s_memtime();
        pR = R;
        pmax = wave_max_all(cnt);
      }
      if constexpr (PROD) {  // stages from the producer wave; the group's last is freed at its end
        k3p_consume(wl, flags, S, R - 1u, h, polls, spin);
        S += (4u * (R - 1u) + 15u) / 16u;
      } else {
        md5_coop<16>(wl, src, h, L.next + 1u, R - 1u);
      }
      if (probe && first) {
        pc2 = __builtin_amdgcn_s_memtime();
        pt2 = __builtin_amdgcn_s_memrealtime();
      }
      // A group that straddles two order bins mixes counts (e.g. 4,229 and
      // 4,093 blocks): the lanes still holding blocks go on cooperatively
      // while the others shadow the first of them and discard (the lane-mode
      // path would take ~1.5x per block, and such a wave was the launch's
      // last by 120 us: bench --k3-probe).
      uint32_t pos = b0 + R, rem = cnt ? cnt - R : 0u;
      for (int round = 0; round < 4; round++) {
        const uint32_t mx = wave_max_all(rem ? ~rem : 0u);
        if (mx == 0u || ~mx < kCoopMinBudget) break;  // wave-uniform
        const uint32_t R2 = ~mx;
        const bool part_ = rem != 0u;
        const int Lr = __builtin_ctzll(__builtin_amdgcn_ballot_w64(part_));
        const uint64_t s_sh = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(reinterpret_cast<uint64_t>(src) >> 32), Lr) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)reinterpret_cast<uint64_t>(src), Lr);
        const uint32_t p_sh = (uint32_t)__builtin_amdgcn_readlane((int)pos, Lr);
        uint32_t hk[4] = {h[0], h[1], h[2], h[3]};
        md5_coop<16>(wl, part_ ? src : reinterpret_cast<const uint8_t*>(s_sh), hk, part_ ? pos : p_sh, R2);
        if (part_) {
          h[0] = hk[0];
          h[1] = hk[1];
          h[2] = hk[2];
          h[3] = hk[3];
          pos += R2;
          rem -= R2;
        }
      }
      md5_run<PROD ? 4 : HBX_MD5_RING>(src, len, h, pos, rem, finish);
      if constexpr (PROD) k3p_publish(&flags[1], S);  // the LDS is the producer's again
    } else {
      md5_run<PROD ? 4 : HBX_MD5_RING>(src, len, h, b0, cnt, finish);
    }
    if constexpr (!ITEMS) {
      if (finish) {
        *(__attribute__((address_space(1))) u32x4*)L.chp->out = u32x4{h[0], h[1], h[2], h[3]};
        L.chp->next = kChainDone;
      } else if (L.live) {
        *reinterpret_cast<uint4*>(&L.chp->h[0]) = make_uint4(h[0], h[1], h[2], h[3]);
        L.chp->next = b0 + cnt;
      }
    } else {  // the next part may run on another CU: agent-scope stores (see k3_lane)
      if (finish) {
        *(__attribute__((address_space(1))) u32x4*)L.chp->out = u32x4{h[0], h[1], h[2], h[3]};
        __hip_atomic_store(&L.chp->next, kChainDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (L.live && cnt) {
#pragma unroll
        for (int i = 0; i < 4; i++) __hip_atomic_store(&L.chp->h[i], h[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&L.chp->next, b0 + cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (ITEMS) {
      if (part + 1u < Q.parts) k3q_push(Q.qc, Q.q, Q.tag, item + groups);
    }
    first = false;
  }
  if (probe && (threadIdx.x & 63u) == 0u) {
    uint64_t* p = probe + 8u * (blockIdx.x * (kK3Threads / 64) + wave);
    // hardware placement: HW_ID (wave, SIMD, CU, SH, SE) and XCC_ID
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xfu;
    p[0] = pt0;
    p[1] = pt1 | ((uint64_t)xcc << 56);
    p[2] = __builtin_amdgcn_s_memrealtime();
    p[3] = (uint64_t)min(pR, 0xffffu) | ((uint64_t)min(pmax, 0xffffu) << 16) | ((uint64_t)hw << 32);
    // the first group's cooperative phase (R - 1 blocks of each chain):
    // shader cycles (s_memtime) and 100 MHz ticks, so cycles per block and the
    // clock follow (bench.py's lifetime decomposition)
    p[4] = pc1;
    p[5] = pc2;
    p[6] = pt2;
    p[7] = (pR ? pR - 1u : 0u) | ((uint64_t)polls << 32);  // + the launch's stage-wait polls (s_sleep 1 each)
  }
  if (started && tslot && (threadIdx.x & 63u) == 0u) {
    const uint32_t tk = __hip_atomic_fetch_add(started + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == t_last) tslot[1] = __builtin_amdgcn_s_memrealtime();
  }
}


// One wave per SIMD: 4-block stages, two register sets, an 8-block lane ring
// (VGPR + AGPR, 346 registers, no scratch).
extern "C" __global__ __launch_bounds__(kK3Threads, 1) void hbx_k3_block_md5(
    const OrderEntry* __restrict__ order, const uint32_t* __restrict__ n_order, uint32_t budget,
    uint32_t* __restrict__ started, uint32_t t_first, uint32_t t_last, uint64_t* __restrict__ tslot,
    uint64_t* __restrict__ probe) {
  __shared__ __attribute__((aligned(16))) uint8_t k3_lds[kK3Threads / 64][kK3WaveLds];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  k3_body<false>(k3_lds[wave], order, n_order, budget, started, t_first, t_last, tslot, probe);
}

// K3P: the same with a producer wave per MD5 wave (waves 4-7 load for waves
// 0-3 of the workgroup; 512 threads, one workgroup per CU).  Same arguments,
// results and launch accounting (only the MD5 waves count in started[1]).
constexpr int kK3PThreads = 512;
extern "C" __global__ __launch_bounds__(kK3PThreads, 1) void hbx_k3p_block_md5(
    const OrderEntry* __restrict__ order, const uint32_t* __restrict__ n_order, uint32_t budget,
    uint32_t* __restrict__ started, uint32_t t_first, uint32_t t_last, uint64_t* __restrict__ tslot,
    uint64_t* __restrict__ probe, uint32_t psets) {
  // psets: producer register sets (2 or 3) | 0x100 for the spinning stage wait
  const bool spin = (psets & 0x100u) != 0u;
  psets &= 0xffu;
  __shared__ __attribute__((aligned(16))) uint8_t k3_lds[4][kK3WaveLds];
  __shared__ uint32_t k3_flags[4][2];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t pair = wave & 3u;
  if (threadIdx.x < 8u) k3_flags[threadIdx.x >> 1][threadIdx.x & 1u] = 0u;
  __syncthreads();
  if (wave < 4u) {
    k3_body<true>(k3_lds[pair], order, n_order, budget, started, t_first, t_last, tslot, probe, k3_flags[pair],
                  K3Queue{}, spin);
  } else {
    __builtin_amdgcn_s_setprio(2);
    if (psets == 3u)
      k3p_producer<3>(k3_lds[pair], k3_flags[pair], order, n_order, budget, blockIdx.x * 4u + pair, gridDim.x * 4u);
    else
      k3p_producer<2>(k3_lds[pair], k3_flags[pair], order, n_order, budget, blockIdx.x * 4u + pair, gridDim.x * 4u);
  }
}

// K3Q: K3P with the launch's work handed out as items (parts of a group's
// slice) through a queue (see k3q_pop).  qc = the order slot's head and tail
// (octl + 1, zeroed by the plan), q its entries, tag = launch index + 1,
// parts = items per group (>= 1), err = a word set if a wave ever gave up
// waiting for an item (never expected; the results are then wrong).
extern "C" __global__ __launch_bounds__(kK3PThreads, 1) void hbx_k3q_block_md5(
    const OrderEntry* __restrict__ order, const uint32_t* __restrict__ n_order, uint32_t budget,
    uint32_t* __restrict__ started, uint32_t t_first, uint32_t t_last, uint64_t* __restrict__ tslot,
    uint64_t* __restrict__ probe, uint32_t* __restrict__ qc, uint64_t* __restrict__ q, uint32_t tag, uint32_t parts,
    uint32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t k3_lds[4][kK3WaveLds];
  __shared__ uint32_t k3_flags[4][4];  // [pair]: stages written, stages freed, item, items announced
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t pair = wave & 3u;
  if (threadIdx.x < 16u) k3_flags[threadIdx.x >> 2][threadIdx.x & 3u] = 0u;
  __syncthreads();
  if (wave < 4u) {
    k3_body<true, true>(k3_lds[pair], order, n_order, budget, started, t_first, t_last, tslot, probe, k3_flags[pair],
                        K3Queue{qc, q, tag, parts, err});
  } else {
    __builtin_amdgcn_s_setprio(2);
    const uint32_t per_part = budget == kBudgetAll ? kBudgetAll : (budget + parts - 1u) / parts;
    k3q_producer(k3_lds[pair], k3_flags[pair], order, n_order, budget, parts, per_part);
  }
}

// K1 gate (scan stream, just before a batch's K1): holds the K1 back until
// every workgroup of the K3 launch issued in the same submit has been
// dispatched (K3's workgroups count themselves into *started), so K3's MD5
// waves take their CUs before K1's 512 workgroups compete for them; K1 then
// fills the CUs K3 leaves free.  One wave; lane 0 polls with vector loads.
// The wait is bounded (limit in 100 MHz ticks of s_memrealtime): a gate
// that times out only delays its K1.
// With meta (round 6, c->gate_meta): the kernel first copies the batch's
// meta block from its pinned staging buffer (hbx_meta_fetch's loads, below),
// so the scan stream runs one kernel fewer per step (one hand-off less before
// K1: the scan loop sets the step at 8 files per GPU); only workgroup 0's
// first lane polls, and only if `poll`.
__device__ __forceinline__ void meta_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t* p = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(src + i));
    uint4 v;
    v.x = __hip_atomic_load(p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.z = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.w = __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    dst[i] = v;
  }
}
extern "C" __global__ __launch_bounds__(256) void hbx_k1_gate_meta(const uint32_t* __restrict__ started,
                                                                   uint32_t target, uint32_t limit,
                                                                   uint32_t poll, const uint4* __restrict__ msrc,
                                                                   uint4* __restrict__ mdst, uint32_t n16) {
  meta_copy(msrc, mdst, n16);
  if (!poll || blockIdx.x != 0 || threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = __hip_atomic_load(started, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((int32_t)(v - target) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)limit) break;
    __builtin_amdgcn_s_sleep(2);
  }
}
extern "C" __global__ __launch_bounds__(64) void hbx_k1_gate(const uint32_t* __restrict__ started,
                                                              uint32_t target, uint32_t limit) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = __hip_atomic_load(started, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if ((int32_t)(v - target) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)limit) break;
    __builtin_amdgcn_s_sleep(2);
  }
}

// A batch's meta block (file offsets, lengths, slice and cut bases, K1's
// tiles) from the pinned host staging buffer into device memory, read over
// PCIe by this kernel on the scan stream in place of hipMemcpyAsync: an SDMA
// copy between two kernels of one stream waits ~17 us for the previous K1's
// completion signal and the next K1 ~25 us for the copy's, ~50 us per step
// on the scan loop (profiles/r05k/scan_gaps.txt: 8 files per GPU, 500 us
// per step); a kernel follows the previous kernel directly.  `n` 16-B words.
// The staging buffer is reused by later batches of the same pool slot, so the
// reads are system-scope (coherent with the host's writes, never a line a
// cache kept from an earlier batch).
extern "C" __global__ __launch_bounds__(256) void hbx_meta_fetch(const uint4* __restrict__ src,
                                                                 uint4* __restrict__ dst, uint32_t n) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    uint32_t* p = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(src + i));
    uint4 v;
    v.x = __hip_atomic_load(p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.z = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    v.w = __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    dst[i] = v;
  }
}

// A finished batch's results (d_res) into its pinned host buffer, written by
// this kernel on the result stream in place of hipMemcpyAsync (c->d2h_kernel):
// an SDMA copy call held the submitting host thread ~7 ms once in a while
// (profiles/r05ay: the D2H call inside finalize_batch).  `n` 16-B words; the
// stores go over PCIe and are made visible to the host before the completion
// event by a system-scope fence.
extern "C" __global__ __launch_bounds__(256) void hbx_result_push(const uint4* __restrict__ src,
                                                                  uint4* __restrict__ dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
    dst[i] = src[i];
  __threadfence_system();
}

// ContentBlockID (store.go:187-196), one wave per file.  The file's ids are
// staged into LDS by all 64 lanes at once (kK4Window per round trip) and the
// chain-block message is generated from there: the ids are read twice
// (once as BlockIDs, once as FileChainBlock links), and a lane fetching them
// one 16-B load per step paid a dependent memory round trip per message block,
// which beside K1's HBM stream made K4 take 0.2-0.45 ms for 8 files.  Every
// lane runs the same MD5 (uniform control flow); lane 0 stores it.
constexpr uint32_t kK4Window = 1024u;  // ids per LDS window (16 KiB); `window` <= this (tests shrink it)

extern "C" __global__ __launch_bounds__(64) void hbx_k4_content_id(
    uint32_t n_files, const uint64_t* __restrict__ cut_base, const uint32_t* __restrict__ cut_count,
    const uint32_t* __restrict__ ids, uint32_t* __restrict__ content_ids,
    int32_t* __restrict__ content_type, uint32_t window) {
  __shared__ uint4 win[kK4Window];
  const uint32_t f = blockIdx.x;
  if (f >= n_files) return;
  const uint32_t k = cut_count[f];
  const uint4* id = reinterpret_cast<const uint4*>(ids) + cut_base[f];
  uint4* co = reinterpret_cast<uint4*>(content_ids) + f;
  if (k <= 1u) {
    if (threadIdx.x == 0) {
      *co = k ? id[0] : make_uint4(0u, 0u, 0u, 0u);
      content_type[f] = k ? 2 : 0;  // ContentTypeFileData / none
    }
    return;
  }
  uint32_t w0 = 0xFFFFFFFFu;  // first id index in the window (none yet)
  auto get = [&](uint32_t i) -> uint4 {
    if (i < w0 || i - w0 >= window) {  // uniform: every lane asks for the same word
      __syncthreads();
      for (uint32_t t = threadIdx.x; t < window && i + t < k; t += 64u) win[t] = id[i + t];
      __syncthreads();
      w0 = i;
    }
    return win[i - w0];
  };
  // Message words (little-endian u32 view of the hashed byte stream):
  //   BE32(k) | id_1..id_k | BE32(8+32k) | "fchn" | BE32(k) | (id_i | 0^16)*k
  const uint32_t nw = 12u * k + 4u;
  const uint32_t T = 4u * nw;
  const uint32_t nblk = (T + 9u + 63u) / 64u;
  uint32_t h[4];
  md5_init(h);
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t j = 16u * b + (uint32_t)i;
      uint32_t v;
      if (j == 0u) {
        v = bswap32(k);
      } else if (j <= 4u * k) {
        const uint4 q = get((j - 1u) >> 2);
        const uint32_t r = (j - 1u) & 3u;
        v = r == 0 ? q.x : r == 1 ? q.y : r == 2 ? q.z : q.w;
      } else if (j == 4u * k + 1u) {
        v = bswap32(8u + 32u * k);
      } else if (j == 4u * k + 2u) {
        v = bswap32(0x6663686Eu);
      } else if (j == 4u * k + 3u) {
        v = bswap32(k);
      } else if (j < nw) {
        const uint32_t t = j - (4u * k + 4u);
        const uint32_t r = t & 7u;
        if (r < 4u) {
          const uint4 q = get(t >> 3);
          v = r == 0 ? q.x : r == 1 ? q.y : r == 2 ? q.z : q.w;
        } else {
          v = 0u;
        }
      } else if (j == nw) {
        v = 0x80u;
      } else {
        v = 0u;
      }
      m[i] = v;
    }
    if (b + 1 == nblk) {
      const uint64_t bits = (uint64_t)T * 8ull;
      m[14] = (uint32_t)bits;
      m[15] = (uint32_t)(bits >> 32);
    }
    md5_compress(h, m);
  }
  if (threadIdx.x == 0) {
    *co = make_uint4(h[0], h[1], h[2], h[3]);
    content_type[f] = 3;  // ContentTypeFileChain
  }
}

// Plain MD5 over a device buffer (used by hbx_block_id for arbitrary blocks
// with links: the host lays out BE32(n)|links|BE32(len) in front).
extern "C" __global__ __launch_bounds__(64) void hbx_k5_md5_raw(const uint8_t* __restrict__ msg,
                                                                 uint32_t n, uint32_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  uint32_t h[4];
  md5_init(h);
  const uint32_t nblk = (n + 9u + 63u) / 64u;
  for (uint32_t b = 0; b < nblk; b++) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      uint32_t v = 0u;
#pragma unroll
      for (int y = 0; y < 4; y++) {
        const uint32_t p = 64u * b + 4u * (uint32_t)i + (uint32_t)y;
        const uint32_t by = p < n ? msg[p] : (p == n ? 0x80u : 0u);
        v |= by << (8 * y);
      }
      m[i] = v;
    }
    if (b + 1 == nblk) {
      const uint64_t bits = (uint64_t)n * 8ull;
      m[14] = (uint32_t)bits;
      m[15] = (uint32_t)(bits >> 32);
    }
    md5_compress(h, m);
  }
  out[0] = h[0];
  out[1] = h[1];
  out[2] = h[2];
  out[3] = h[3];
}

// ------------------------------------------------------------ K6 verify --
// Batched HashboxBlock.HashData / VerifyBlock (pkg/core/block.go:96-111,
// 152-174) for uncompressed blocks: lane per block, message =
// BE32(n_links) || links || BE32(len) || data.  The message blocks that hold
// prefix bytes are built byte by byte (a short message entirely so); the
// data-only rest runs through the streaming path (md5_run, md5_tail), whose
// framing is an 8-byte prefix, on a virtual start shifted back by
// (prefix - 8) bytes: from block ceil(prefix/64) on, every byte it reads lies
// inside the block's data.
struct VerifyDesc {
  uint64_t src;      // device address of the block's data
  uint64_t links;    // device address of its n_links 16-byte link IDs
  uint32_t len;      // data bytes
  uint32_t n_links;
  uint64_t pad;
};
static_assert(sizeof(VerifyDesc) == 32, "descriptor layout shared with the host");

namespace {
__device__ __forceinline__ uint32_t k6_byte(uint64_t o, uint32_t nl, uint32_t len, uint32_t p, uint64_t T,
                                            const uint8_t* links, const uint8_t* data) {
  if (o < 4u) return (nl >> (8u * (3u - (uint32_t)o))) & 0xffu;
  if (o < 4u + 16ull * nl) return links[o - 4u];
  if (o < p) return (len >> (8u * (3u - (uint32_t)(o - 4u - 16ull * nl)))) & 0xffu;
  if (o < T) return data[o - p];
  return o == T ? 0x80u : 0u;
}
}  // namespace

// One wave per workgroup (the waves of a launch spread over the CUs, as K3's
// spread placement); blocks arrive sorted longest first, so a wave's 64
// chains are about equally long and advance their common count through the
// cooperative path.
extern "C" __global__ __launch_bounds__(64, 1) void hbx_k6_hash_blocks(
    const VerifyDesc* __restrict__ desc, uint32_t n, const uint8_t* __restrict__ zeros,
    uint32_t* __restrict__ ids, const uint32_t* __restrict__ expect, uint8_t* __restrict__ ok) {
  __shared__ __attribute__((aligned(16))) uint8_t k6_lds[kCoopWaveLds];
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  const bool active = i < n;
  const VerifyDesc v = desc[active ? i : 0u];  // n >= 1: idle lanes shadow block 0 and store nothing
  const uint32_t len = v.len, nl = v.n_links;
  const uint32_t p = 8u + 16u * nl;       // prefix bytes
  const uint64_t T = (uint64_t)len + p;   // message bytes (< 2^32 - 128, checked by the host)
  const uint32_t nfull = (uint32_t)(T >> 6);
  const uint32_t hb = (p + 63u) >> 6;     // message blocks holding prefix bytes
  const bool fast = nfull >= hb;          // the tail holds no prefix byte
  const uint32_t nslow = fast ? hb : (uint32_t)((T + 8u) >> 6) + 1u;
  const uint8_t* data = reinterpret_cast<const uint8_t*>(v.src);
  const uint8_t* links = reinterpret_cast<const uint8_t*>(v.links);
  uint32_t h[4];
  md5_init(h);
  for (uint32_t b = 0; b < nslow; b++) {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const uint64_t o = 64ull * b + 4u * (uint32_t)j;
      m[j] = k6_byte(o, nl, len, p, T, links, data) | (k6_byte(o + 1u, nl, len, p, T, links, data) << 8) |
             (k6_byte(o + 2u, nl, len, p, T, links, data) << 16) |
             (k6_byte(o + 3u, nl, len, p, T, links, data) << 24);
    }
    if (!fast && b + 1u == nslow) {
      const uint64_t bits = T * 8ull;
      m[14] = (uint32_t)bits;
      m[15] = (uint32_t)(bits >> 32);
    }
    md5_compress(h, m);
  }
  // data-only full blocks (wave-uniform call; a lane with none streams an
  // empty range over a zero page), then the tail
  const uint32_t cnt = fast ? nfull - hb : 0u;
  const uint8_t* vs = data - (p - 8u);
  // every lane is at block hb >= 1 of its message: the wave's smallest
  // count R goes through the cooperative loads (idle lanes shadow block 0,
  // the longest), the per-lane remainder through the lane path
  const uint32_t R = ~wave_max_all(active ? ~cnt : 0u);
  const uint32_t Rc = R >= kCoopMinBudget ? R : 0u;  // wave-uniform
  if (Rc) md5_coop<16>(k6_lds, vs, h, hb, Rc);
  const uint32_t rest = cnt - Rc;
  md5_run<>(rest ? vs : zeros + 64, rest ? len + p - 8u : 0u, h, rest ? hb + Rc : 1u, rest, false);
  if (fast) md5_tail(vs, len + p - 8u, h, true);
  if (active) {
    *reinterpret_cast<uint4*>(ids + 4u * i) = make_uint4(h[0], h[1], h[2], h[3]);
    if (expect)
      ok[i] = (uint8_t)(h[0] == expect[4u * i] && h[1] == expect[4u * i + 1u] && h[2] == expect[4u * i + 2u] &&
                        h[3] == expect[4u * i + 3u]);
  }
}

// Pipelined VerifyBlock (hbx_verify_submit_device): thread per block.  A
// block's message is BE32(n) || links || BE32(len) || data; K3's chains hash
// BE32(0) || BE32(len') || chunk'.  With chunk' = data - 16n and
// len' = len + 16n the two agree from the first message block that holds no
// prefix byte on, so this kernel hashes the prefix blocks byte by byte (as
// K6) and hands the rest to the time-sliced K3 pipeline as an ordinary chain
// starting at that block.  A block whose last partial message block still
// holds prefix bytes is finished here.  Blocks without links are plain K3
// chains from block 0.
extern "C" __global__ __launch_bounds__(256) void hbx_k6p_verify_chains(
    const VerifyDesc* __restrict__ desc, uint32_t n, uint32_t* __restrict__ ids, Chain* __restrict__ run,
    OrderEntry* __restrict__ fresh, uint32_t* __restrict__ cnt) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const VerifyDesc v = desc[i];
  const uint32_t len = v.len, nl = v.n_links;
  Chain ch;
  ch.out = reinterpret_cast<uint64_t>(ids + 4u * i);
  ch.pad = 0ull;
  uint32_t rem;
  if (nl == 0u) {
    ch.src = v.src;
    ch.len = len;
    ch.next = 0u;
    md5_init(ch.h);
    rem = ((len + 8u) >> 6) + 1u;
  } else {
    const uint32_t p = 8u + 16u * nl;
    const uint64_t T = (uint64_t)len + p;
    const uint32_t nfull = (uint32_t)(T >> 6);
    const uint32_t hb = (p + 63u) >> 6;
    const bool fast = nfull >= hb;
    const uint32_t nslow = fast ? hb : (uint32_t)((T + 8u) >> 6) + 1u;
    const uint8_t* data = reinterpret_cast<const uint8_t*>(v.src);
    const uint8_t* links = reinterpret_cast<const uint8_t*>(v.links);
    uint32_t h[4];
    md5_init(h);
    for (uint32_t b = 0; b < nslow; b++) {
      uint32_t m[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint64_t o = 64ull * b + 4u * (uint32_t)j;
        m[j] = k6_byte(o, nl, len, p, T, links, data) | (k6_byte(o + 1u, nl, len, p, T, links, data) << 8) |
               (k6_byte(o + 2u, nl, len, p, T, links, data) << 16) |
               (k6_byte(o + 3u, nl, len, p, T, links, data) << 24);
      }
      if (!fast && b + 1u == nslow) {
        const uint64_t bits = T * 8ull;
        m[14] = (uint32_t)bits;
        m[15] = (uint32_t)(bits >> 32);
      }
      md5_compress(h, m);
    }
    if (!fast) {  // finished here
      *reinterpret_cast<uint4*>(ids + 4u * i) = make_uint4(h[0], h[1], h[2], h[3]);
      return;
    }
    ch.src = v.src - (p - 8u);
    ch.len = len + p - 8u;
    ch.next = hb;
    ch.h[0] = h[0];
    ch.h[1] = h[1];
    ch.h[2] = h[2];
    ch.h[3] = h[3];
    rem = nfull - hb + 1u;
  }
  const uint32_t slot = atomicAdd(cnt, 1u);
  run[slot] = ch;
  OrderEntry o;
  o.chain = reinterpret_cast<uint64_t>(run + slot);
  o.rem = rem;
  o.pad = 0u;
  fresh[slot] = o;
}

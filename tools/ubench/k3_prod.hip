// K3's cooperative MD5 path with and without a producer wave (verdict r04
// item 1): does taking the global loads and the LDS staging out of the MD5
// wave's instruction stream bring a block from ~1,560 cycles toward the
// 1,312 of the bare VALU chain?
//
//   base   the shipped path: hbx_kernels.hip's md5_block_at + md5_coop<16>,
//          one 256-thread workgroup per CU (one MD5 wave per SIMD), each wave
//          loading, staging and hashing its own 64 chains.
//   prod   512-thread workgroups: waves 0-3 hash (one per SIMD), waves 4-7
//          load: producer p issues the 16 global loads of each 4-block stage
//          of consumer p's 64 chains, writes the 272-B LDS rows and publishes
//          the stage through an LDS counter; the consumer waits on that
//          counter, reads its row (4 ds_read_b128 per block), hashes, and
//          frees the stage through a second counter.  No s_barrier.
//
// Chains: 32,768 at random byte offsets over a large buffer (the residency of
// 33 resident 8 GiB batches), R blocks each.  Both kernels must produce the
// same digests.  Reported per case: launch ms, GB/s, the in-kernel clock
// (s_memtime / s_memrealtime) and cycles per block per chain; alone and beside
// a K1-like nontemporal streamer on the CUs left free.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../hashbox_amd/csrc -o k3_prod k3_prod.hip
#include "../../hashbox_amd/csrc/hbx_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

constexpr uint32_t kLen = 0x7fffffffu;  // framing length of block 0 (the data is what it is)

__device__ __forceinline__ void stamp(uint64_t* st, int k) {
  if ((threadIdx.x & 63u) == 0u) {
    st[2 * k] = __builtin_amdgcn_s_memtime();
    st[2 * k + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// ----------------------------------------------------------------- base --
__global__ __launch_bounds__(256, 1) void k3_base(const uint64_t* __restrict__ addr, uint32_t R,
                                                   u32x4* __restrict__ out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][kCoopWaveLds];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t gw = blockIdx.x * 4u + wave;
  uint64_t* st = stamps + 8u * gw;
  __builtin_amdgcn_s_setprio(3);
  stamp(st, 0);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(addr[64u * gw + lane]);
  uint32_t h[4];
  md5_init(h);
  md5_block_at(c, kLen, h, 0u);
  md5_coop<16>(lds[wave], c, h, 1u, R - 1u);
  out[64u * gw + lane] = u32x4{h[0], h[1], h[2], h[3]};
  stamp(st, 1);
  if ((threadIdx.x & 63u) == 0u) st[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
}

// ----------------------------------------------------------------- prod --
// The product's K3P pair code (hbx_kernels.hip k3p_consume / k3p_produce) on
// one group per pair: blocks 1..R-1 of the wave's 64 chains.
template <int PRIO_P>
__global__ __launch_bounds__(512, 1) void k3_prod(const uint64_t* __restrict__ addr, uint32_t R,
                                                   u32x4* __restrict__ out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][kCoopWaveLds];
  __shared__ uint32_t flags[4][2];  // [pair][0] stages written, [pair][1] stages freed
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t pair = wave & 3u;
  if (threadIdx.x < 8u) flags[threadIdx.x >> 1][threadIdx.x & 1u] = 0u;
  __syncthreads();
  const uint32_t gw = blockIdx.x * 4u + pair;
  const uint8_t* c = reinterpret_cast<const uint8_t*>(addr[64u * gw + lane]);
  if (wave < 4u) {
    uint64_t* st = stamps + 8u * gw;
    __builtin_amdgcn_s_setprio(3);
    stamp(st, 0);
    uint32_t h[4];
    md5_init(h);
    md5_block_at(c, kLen, h, 0u);
    k3p_consume(lds[pair], flags[pair], 0u, R - 1u, h);
    out[64u * gw + lane] = u32x4{h[0], h[1], h[2], h[3]};
    stamp(st, 1);
    if (lane == 0u) st[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  } else {
    __builtin_amdgcn_s_setprio(PRIO_P);
    k3p_produce(lds[pair], flags[pair], 0u, reinterpret_cast<uint64_t>(c) + 64ull - 8ull, R - 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0u) stamps[8u * gw + 5] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
  }
}

// ------------------------------------------------------------ floors --
// The MD5 wave's cost without the memory side: `cons` hashes the LDS stages
// (4 ds_read_b128 per block, k3p_consume) with every stage published up front
// and no producer; `valu` compresses blocks from registers only (the bare
// VALU chain of the compiled md5_compress).  Digests are not compared.
template <int MODE>
__global__ __launch_bounds__(256, 1) void k3_floor(const uint64_t* __restrict__ addr, uint32_t R,
                                                    u32x4* __restrict__ out, uint64_t* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][kCoopWaveLds];
  __shared__ uint32_t flags[4][2];
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  if (threadIdx.x < 8u) flags[threadIdx.x >> 1][threadIdx.x & 1u] = (threadIdx.x & 1u) ? 0u : 0x7fffffffu;
  for (uint32_t i = threadIdx.x; i < 4u * kCoopWaveLds / 4u; i += 256u)
    reinterpret_cast<uint32_t*>(&lds[0][0])[i] = i * 0x9e3779b9u;
  __syncthreads();
  const uint32_t gw = blockIdx.x * 4u + wave;
  uint64_t* st = stamps + 8u * gw;
  __builtin_amdgcn_s_setprio(3);
  uint32_t h[4];
  md5_init(h);
  h[0] ^= (uint32_t)addr[64u * gw + lane];
  stamp(st, 0);
  if constexpr (MODE == 0) {
    k3p_consume(lds[wave], flags[wave], 0u, R, h);
  } else {
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = h[j & 3] * (uint32_t)(j + 1);
    for (uint32_t b = 0; b < R; b++) {
      m[b & 15u] ^= b;  // (a runtime index: the block's words change every block)
      md5_compress(h, m);
    }
  }
  stamp(st, 1);
  out[64u * gw + lane] = u32x4{h[0], h[1], h[2], h[3]};
  if (lane == 0u) st[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
}

// ------------------------------------------------------------- streamer --
// 1024-thread workgroups holding 128 KiB of (unused) LDS, like K1: they cannot
// share a CU with a K3 workgroup.
__global__ __launch_bounds__(1024) void stream_read(const u32x4* __restrict__ p, uint64_t n16, uint32_t reps,
                                                    uint32_t* __restrict__ sink) {
  extern __shared__ uint32_t pad_lds[];
  if (reps == 0xffffffffu) pad_lds[threadIdx.x] = 0u;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint32_t r = 0; r < reps; r++)
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 3 * stride < n16; i += 4 * stride)
      acc ^= __builtin_nontemporal_load(p + i) ^ __builtin_nontemporal_load(p + i + stride) ^
             __builtin_nontemporal_load(p + i + 2 * stride) ^ __builtin_nontemporal_load(p + i + 3 * stride);
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) sink[0] = x;
}

__global__ void fill(uint32_t* p, uint64_t n, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9e3779b97f4a7c15ull + seed;
    x ^= x >> 31;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 29;
    p[i] = (uint32_t)x;
  }
}

int main(int argc, char** argv) {
  const uint64_t big = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 64ull) << 30;
  const uint32_t S = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 10) : 32768u;  // chains
  const uint32_t R = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 10) : 4096u;   // blocks per chain
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  const uint64_t sbytes = 8ull << 30;
  uint8_t *d_big = nullptr, *d_s = nullptr;
  CK(hipMalloc(&d_big, big + (1u << 20)));
  CK(hipMalloc(&d_s, sbytes));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)d_big, (big + (1u << 20)) / 4, 7u);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)d_s, sbytes / 4, 9u);
  CK(hipDeviceSynchronize());
  std::mt19937_64 rng(11);
  const uint64_t span = 64ull * R + 256;
  std::vector<uint64_t> h(S);
  for (auto& a : h) a = (uint64_t)d_big + 64 + rng() % (big - span - 64);
  uint64_t* d_addr = nullptr;
  u32x4 *d_outa = nullptr, *d_outb = nullptr;
  uint64_t* d_st = nullptr;
  uint32_t* d_sink = nullptr;
  const uint32_t waves = S / 64u, wgs = waves / 4u;
  CK(hipMalloc(&d_addr, 8ull * S));
  CK(hipMalloc(&d_outa, 16ull * S));
  CK(hipMalloc(&d_outb, 16ull * S));
  CK(hipMalloc(&d_st, 64ull * waves));
  CK(hipMalloc(&d_sink, 64));
  CK(hipMemcpy(d_addr, h.data(), 8ull * S, hipMemcpyHostToDevice));
  hipStream_t sk, ss;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint64_t> hs(8ull * waves);
  printf("# %u chains x %u blocks (%.2f GB per launch), buffer %.0f GiB, %u workgroups\n", S, R,
         64.0 * R * S / 1e9, big / 1073741824.0, wgs);
  printf("# kernel, beside, ms, GB/s, clock_GHz(med), cycles_per_block(med wave), p10, p90, workgroups whose MD5 waves hold 4 distinct SIMDs\n");
  const char* names[] = {"base", "prod_p0", "prod_p2", "floor_cons", "floor_valu"};
  for (int kind = 0; kind < 5; kind++) {
    for (int beside = 0; beside < 2; beside++) {
      float best = 1e30f;
      for (int r = 0; r < reps; r++) {
        CK(hipMemset(d_st, 0, 64ull * waves));
        CK(hipEventRecord(e0, sk));
        u32x4* o = kind == 0 ? d_outa : d_outb;
        if (kind == 0)
          hipLaunchKernelGGL(k3_base, dim3(wgs), dim3(256), 0, sk, d_addr, R, o, d_st);
        else if (kind == 1)
          hipLaunchKernelGGL(k3_prod<0>, dim3(wgs), dim3(512), 0, sk, d_addr, R, o, d_st);
        else if (kind == 2)
          hipLaunchKernelGGL(k3_prod<2>, dim3(wgs), dim3(512), 0, sk, d_addr, R, o, d_st);
        else if (kind == 3)
          hipLaunchKernelGGL(k3_floor<0>, dim3(wgs), dim3(256), 0, sk, d_addr, R, o, d_st);
        else
          hipLaunchKernelGGL(k3_floor<1>, dim3(wgs), dim3(256), 0, sk, d_addr, R, o, d_st);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, sk));
        if (beside) {
          usleep(200);
          hipLaunchKernelGGL(stream_read, dim3(256 - std::min(wgs, 255u)), dim3(1024), 128 * 1024, ss,
                             (const u32x4*)d_s, sbytes / 16, 4u, d_sink);
          CK(hipGetLastError());
        }
        CK(hipDeviceSynchronize());
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
      }
      CK(hipMemcpy(hs.data(), d_st, 64ull * waves, hipMemcpyDeviceToHost));
      std::vector<double> cpb, clk;
      int simd_ok = 0;
      for (uint32_t w = 0; w < waves; w++) {
        const uint64_t* s = &hs[8ull * w];
        const double cyc = (double)(s[2] - s[0]), rt = (double)(s[3] - s[1]);
        if (rt > 0) {
          cpb.push_back(cyc / R);
          clk.push_back(cyc / rt * 0.1);
        }
      }
      // the MD5 waves of each workgroup on four distinct SIMDs (HW_ID)
      for (uint32_t wg = 0; wg < wgs; wg++) {
        uint32_t m = 0;
        for (uint32_t k = 0; k < 4u; k++) m |= 1u << (((uint32_t)hs[8ull * (4u * wg + k) + 4] >> 4) & 3u);
        simd_ok += m == 15u ? 1 : 0;
      }
      std::sort(cpb.begin(), cpb.end());
      std::sort(clk.begin(), clk.end());
      auto q = [](const std::vector<double>& v, double f) { return v.empty() ? 0.0 : v[(size_t)(f * (v.size() - 1))]; };
      printf("%s, %d, %.3f, %.1f, %.3f, %.1f, %.1f, %.1f, %d/%u\n", names[kind], beside, best,
             64.0 * R * S / (best * 1e6), q(clk, 0.5), q(cpb, 0.5), q(cpb, 0.1), q(cpb, 0.9), simd_ok, wgs);
      fflush(stdout);
    }
    if (kind > 0 && kind < 3) {
      std::vector<u32x4> a(S), b(S);
      CK(hipMemcpy(a.data(), d_outa, 16ull * S, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), d_outb, 16ull * S, hipMemcpyDeviceToHost));
      uint32_t bad = 0;
      for (uint32_t i = 0; i < S; i++)
        bad += (a[i].x != b[i].x || a[i].y != b[i].y || a[i].z != b[i].z || a[i].w != b[i].w) ? 1u : 0u;
      printf("# %s vs base: %u of %u digests differ\n", names[kind], bad, S);
      if (bad) return 2;
    }
  }
  return 0;
}

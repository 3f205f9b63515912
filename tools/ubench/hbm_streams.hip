// K3's memory side without its MD5: how fast HBM serves the access pattern of
// the cooperative chain loads, alone and beside a K1-like sequential reader.
//
//   coop      S streams (chains) at exact byte addresses spread over a large
//             buffer, 64 per wave, one wave per SIMD (256-thread workgroups,
//             34 KiB of LDS per wave as in K3).  Per stage every chain
//             advances 256 B: 16 global_load_dwordx4 of 4 chains x 256 B each
//             (two register sets in flight), staged into LDS rows of 272 B,
//             read back by the lane owning the row (4 ds_read_b128 per 64 B)
//             and folded with one v_xor per word instead of an MD5 block.
//   stream    a grid-stride nontemporal read of another buffer (K1's HBM
//             traffic without its scan), on a second stream, sized to outlast
//             the coop launch.
//
// Reported: the coop launch's time and GB/s alone and beside the streamer (and
// the streamer's own rate while it overlaps), for several chain counts; then
// the same with the stage loads only (no LDS round trip).
// hipcc --offload-arch=gfx950 -O3 -o hbm_streams hbm_streams.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iterator>
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;

constexpr int kG = 16;                      // granules of 16 B per chain per stage (4 blocks)
constexpr uint32_t kC = 64u / kG;           // chains per load instruction
constexpr uint32_t kRow = 16u * kG + 16u;   // 272 B
constexpr uint32_t kHalf = 64u * kRow;
constexpr uint32_t kWaveLds = 2u * kHalf;   // 34 KiB

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const int lo = __builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)v);
  const int hi = __builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// CPW chains per wave (64: K3's layout; 32: the same chains spread over twice
// the waves, i.e. 256 CUs instead of 128, half the LDS rows and half the load
// instructions per stage; lanes >= 32 only help with the loads).
template <bool LDS, int SETS = 2, int CPW = 64>
__global__ __launch_bounds__(256, 1) void coop(const uint64_t* __restrict__ addr, uint32_t stages,
                                               uint32_t* __restrict__ out, uint32_t stride) {
  constexpr int NQ = CPW / (int)kC;  // load instructions per stage
  constexpr uint32_t Half = (uint32_t)CPW * kRow;
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][2u * Half];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint8_t* wl = lds[wave];
  const uint64_t S = addr[(blockIdx.x * 4u + wave) * (uint32_t)CPW + (lane % (uint32_t)CPW)];
  const uint32_t t = lane % kG, sub = lane / kG;
  uint64_t Q[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) Q[q] = shfl64(S, kC * (uint32_t)q + sub) + 16ull * t;
  const uint32_t wr = sub * kRow + 16u * t, rd = lane * kRow;
  u32x4 acc = {0u, 0u, 0u, 0u};
  auto load = [&](u32x4(&G)[NQ], uint32_t st) {
#pragma unroll
    for (int q = 0; q < NQ; q++) G[q] = *(g_u32x4*)(Q[q] + 16ull * kG * stride * st);
  };
  auto write = [&](uint32_t half, const u32x4(&G)[NQ]) {
#pragma unroll
    for (int q = 0; q < NQ; q++) *reinterpret_cast<u32x4*>(wl + wr + half * Half + kC * kRow * (uint32_t)q) = G[q];
  };
  auto use = [&](uint32_t half, const u32x4(&G)[NQ]) {
    if constexpr (LDS) {
      if (CPW == 64 || lane < (uint32_t)CPW) {
#pragma unroll
        for (int k = 0; k < kG; k++) acc ^= *reinterpret_cast<const u32x4*>(wl + rd + half * Half + 16u * k);
      }
    } else {
#pragma unroll
      for (int q = 0; q < NQ; q++) acc ^= G[q];
    }
  };
  u32x4 GA[NQ], GB[NQ];
  load(GA, 0u);
  load(GB, 1u);
  if constexpr (LDS) write(0u, GA);
  else use(0u, GA);
  load(GA, 2u);
  if constexpr (SETS == 2) {
    for (uint32_t s = 0; s + 2u < stages; s += 2u) {
      if constexpr (LDS) write(1u, GB);
      use(0u, GB);
      load(GB, s + 3u);
      if constexpr (LDS) write(0u, GA);
      use(1u, GA);
      load(GA, s + 4u);
    }
  } else {  // three register sets: stages s+1..s+3 in flight while s is used
    u32x4 GC[NQ];
    load(GC, 3u);
    for (uint32_t s = 0; s + 3u < stages; s += 3u) {
      write(1u, GB);
      use(0u, GB);
      load(GB, s + 4u);
      write(0u, GA);
      use(1u, GA);
      load(GA, s + 5u);
      write(1u, GC);
      use(0u, GC);
      load(GC, s + 6u);
    }
  }
  const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x9e3779b9u) out[0] = r;
}

// Eight-block stages: 2 chains x 512 B per load instruction, one LDS stage
// (33 KiB) per wave and the next two in registers, each written right after
// the stage before it is read (hbx_kernels.hip's round-3 STAGE8 experiment).
constexpr int kG8 = 32;
constexpr uint32_t kRow8 = 16u * kG8 + 16u;
__global__ __launch_bounds__(256, 1) void coop8(const uint64_t* __restrict__ addr, uint32_t stages,
                                                uint32_t* __restrict__ out, uint32_t stride) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][64u * kRow8];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint8_t* wl = lds[wave];
  const uint64_t S = addr[(blockIdx.x * 4u + wave) * 64u + lane];
  const uint32_t t = lane % kG8, sub = lane / kG8;
  uint64_t Q[kG8];
#pragma unroll
  for (int q = 0; q < kG8; q++) Q[q] = shfl64(S, 2u * (uint32_t)q + sub) + 16ull * t;
  const uint32_t wr = sub * kRow8 + 16u * t, rd = lane * kRow8;
  u32x4 acc = {0u, 0u, 0u, 0u};
  // stage units of 512 B per chain: stage st covers the 256-B stages 2st, 2st+1
  auto load = [&](u32x4(&G)[kG8], uint32_t st) {
#pragma unroll
    for (int q = 0; q < kG8; q++) G[q] = *(g_u32x4*)(Q[q] + 16ull * kG8 * stride * st);
  };
  auto write = [&](const u32x4(&G)[kG8]) {
#pragma unroll
    for (int q = 0; q < kG8; q++) *reinterpret_cast<u32x4*>(wl + wr + 2u * kRow8 * (uint32_t)q) = G[q];
  };
  auto use = [&]() {
#pragma unroll
    for (int k = 0; k < kG8; k++) acc ^= *reinterpret_cast<const u32x4*>(wl + rd + 16u * k);
  };
  u32x4 GA[kG8], GB[kG8];
  const uint32_t st8 = stages / 2u;
  load(GA, 0u);
  load(GB, 1u);
  write(GA);
  load(GA, 2u);
  for (uint32_t s = 0; s + 2u < st8; s += 2u) {
    use();
    write(GB);
    load(GB, s + 3u);
    use();
    write(GA);
    load(GA, s + 4u);
  }
  const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x9e3779b9u) out[0] = r;
}

// 1024-thread workgroups holding 128 KiB of (unused) dynamic LDS, like K1: they
// cannot share a CU with a coop workgroup, so the two split the CUs as K1 and
// K3 do.  With 64 KiB (the "_shared" cases) one fits beside a 32-chains-per-
// wave coop workgroup (68 KiB) on every CU.
__global__ __launch_bounds__(1024) void stream_read(const u32x4* __restrict__ p, uint64_t n16, uint32_t reps,
                                                    uint32_t* __restrict__ out) {
  extern __shared__ uint32_t pad_lds[];
  if (reps == 0xffffffffu) pad_lds[threadIdx.x] = 0u;  // never: keeps the allocation
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint32_t r = 0; r < reps; r++) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
      acc ^= __builtin_nontemporal_load(p + i) ^ __builtin_nontemporal_load(p + i + stride) ^
             __builtin_nontemporal_load(p + i + 2 * stride) ^ __builtin_nontemporal_load(p + i + 3 * stride);
    }
  }
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9e3779b9u) out[0] = x;
}

int main(int argc, char** argv) {
  const uint64_t big = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 128ull) << 30;  // chain buffer
  const uint64_t sbytes = 8ull << 30;                                                 // streamer buffer
  uint8_t *d_big = nullptr, *d_s = nullptr;
  uint32_t* d_out = nullptr;
  CK(hipMalloc(&d_big, big + (1u << 20)));
  CK(hipMalloc(&d_s, sbytes));
  CK(hipMalloc(&d_out, 64));
  CK(hipMemset(d_big, 0x5a, big + (1u << 20)));
  CK(hipMemset(d_s, 0xa5, sbytes));
  hipStream_t sc, ss;
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
  hipEvent_t c0, c1, s0, s1;
  CK(hipEventCreate(&c0));
  CK(hipEventCreate(&c1));
  CK(hipEventCreate(&s0));
  CK(hipEventCreate(&s1));
  std::mt19937_64 rng(7);
  printf("# chain buffer %.0f GiB; per chain 256 B per stage; coop = one wave per SIMD, 256-thread WGs\n",
         big / 1073741824.0);
  printf("# mode, chains, stages, coop_ms, coop_GBps, streamer_GBps_average (0 = coop alone; the streamer outlasts coop, so its average includes time alone)\n");
  // (mode, placement): coop with 2 or 3 register sets (LDS staging) or 2 sets
  // without LDS; chains at random byte offsets ("rand") or the 64 chains of a
  // wave side by side, 256 B apart, each stage 16 KiB further ("local": the
  // same instruction stream with a streaming footprint of a few pages per wave)
  // "page": the 64 chains of a wave in one 2 MiB page, 32 KiB apart (128
  // stages each): few translations per wave like "local", but every chain's
  // 256 B in a DRAM row of its own like "rand" (TLB reach vs DRAM locality);
  // "rand128" is "rand" over the same 128 stages.
  // "win<M>" (round 6): the 64 chains of a wave at random byte offsets inside a
  // window of M MiB of its own (random, 2 MiB aligned): the translation reach
  // a wave's chains need, between "page" (one 2 MiB page) and "rand" (128 GiB)
  struct Case { const char* name; int sets; bool lds; int place; uint32_t S; int cpw = 64; uint32_t win_mib = 0; };
  // default: round 4, K3's 32,768 chains at 64 per wave (128 CUs, the
  // streamer on the other 128) vs 32 per wave (all 256 CUs, the streamer
  // sharing them with 64 KiB of LDS)
  const Case cases[] = {
      {"coop_lds2_rand", 2, true, 0, 32768u, 64},   {"coop32_lds2_rand", 2, true, 0, 32768u, 32},
      {"coop_lds2_rand", 2, true, 0, 16384u, 64},   {"coop32_lds2_rand", 2, true, 0, 16384u, 32},
  };
  const Case cases_full[] = {
      {"coop_lds2_rand", 2, true, 0, 8192u},   {"coop_lds2_rand", 2, true, 0, 16384u},
      {"coop_lds2_rand", 2, true, 0, 32768u},  {"coop_lds2_rand", 2, true, 0, 65536u},
      {"coop_regs2_rand", 2, false, 0, 32768u}, {"coop_lds3_rand", 3, true, 0, 16384u},
      {"coop_lds3_rand", 3, true, 0, 32768u},  {"coop_lds2_local", 2, true, 1, 16384u},
      {"coop_lds2_local", 2, true, 1, 32768u},  {"coop_lds3_local", 3, true, 1, 32768u},
      {"coop_lds2_page", 2, true, 2, 32768u},   {"coop_lds2_rand128", 2, true, 0, 32768u},
      {"coop8_rand", 8, true, 0, 32768u},        {"coop8_rand", 8, true, 0, 16384u},
      {"coop_lds2_win2", 2, true, 3, 32768u, 64, 2},     {"coop_lds2_win8", 2, true, 3, 32768u, 64, 8},
      {"coop_lds2_win32", 2, true, 3, 32768u, 64, 32},   {"coop_lds2_win128", 2, true, 3, 32768u, 64, 128},
      {"coop_lds2_win512", 2, true, 3, 32768u, 64, 512}, {"coop_lds2_win2048", 2, true, 3, 32768u, 64, 2048},
  };
  // cases_full: the round-3 table (profiles/r03hbms/hbm_streams_sets_local.txt), run by name (argv[2])
  // argv[2] (optional): run only the cases named exactly so, argv[3] only that
  // chain count, without the streamer (for rocprofv3 --pmc passes)
  const char* only = argc > 2 ? argv[2] : nullptr;
  const uint32_t only_s = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 10) : 0u;
  const std::vector<Case> run = only ? std::vector<Case>(std::begin(cases_full), std::end(cases_full))
                                     : std::vector<Case>(std::begin(cases), std::end(cases));
  for (const Case& k : run) {
    if (only && (std::strcmp(k.name, only) != 0 || (only_s && k.S != only_s))) continue;
    const uint32_t S = k.S;
    const bool local = k.place == 1;
    const uint32_t stages = (k.place == 2 || std::strstr(k.name, "128"))
                                ? 128u
                                : (uint32_t)std::min<uint64_t>(4096u, (8ull << 30) / (256ull * S));
    const uint64_t span = 256ull * (stages + 8u) + 64;
    std::vector<uint64_t> h(S);
    for (uint32_t i = 0; i < S; i++) {
      if (k.place == 2) {  // wave w: its own 2 MiB page, chain c at 32 KiB * c
        h[i] = (uint64_t)d_big + (uint64_t)(i / 64u) * (2ull << 20) + 32768ull * (i % 64u) + 8ull;
      } else if (k.place == 3) {  // wave w: a window of win_mib MiB, chains at random offsets in it
        static uint64_t wbase = 0;
        const uint64_t W = (uint64_t)k.win_mib << 20;
        if (i % 64u == 0u) wbase = (rng() % ((big - W - span) >> 21)) << 21;
        h[i] = (uint64_t)d_big + wbase + rng() % (W > span ? W - span : 1ull);
      } else if (local) {  // wave w: chains side by side; stage st of chain c at w*64*span' + 16 KiB*st + 256*c
        const uint64_t w = i / 64u, c = i % 64u;
        h[i] = (uint64_t)d_big + w * 64ull * 256ull * (stages + 8u) + 256ull * c + 8ull;  // (16 KiB per stage: see kernel)
      } else {
        h[i] = (uint64_t)d_big + rng() % (big - span);  // random byte offsets, like chunk starts
      }
    }
    uint64_t* d_addr = nullptr;
    CK(hipMalloc(&d_addr, S * 8ull));
    CK(hipMemcpy(d_addr, h.data(), S * 8ull, hipMemcpyHostToDevice));
    const uint32_t wgs = S / (4u * (uint32_t)k.cpw);
    const bool shared = k.cpw == 32;  // the streamer shares the coop's CUs
    const double bytes = 256.0 * stages * S;
    for (int beside = 0; beside < (only ? 1 : 2); beside++) {
      float best = 1e30f, sms = 0.f;
      for (int rep = 0; rep < 3; rep++) {
        // coop first (its workgroups take their CUs), then the streamer on
        // the CUs left; the streamer outlasts the coop launch
        CK(hipEventRecord(c0, sc));
        const uint32_t stride = local ? 64u : 1u;  // local: stage stride 64 x 256 B = 16 KiB
        if (k.cpw == 32)
          hipLaunchKernelGGL((coop<true, 2, 32>), dim3(wgs), dim3(256), 0, sc, d_addr, stages, d_out, stride);
        else if (k.sets == 8)
          hipLaunchKernelGGL(coop8, dim3(wgs), dim3(256), 0, sc, d_addr, stages, d_out, stride);
        else if (!k.lds)
          hipLaunchKernelGGL((coop<false, 2>), dim3(wgs), dim3(256), 0, sc, d_addr, stages, d_out, stride);
        else if (k.sets == 3)
          hipLaunchKernelGGL((coop<true, 3>), dim3(wgs), dim3(256), 0, sc, d_addr, stages, d_out, stride);
        else
          hipLaunchKernelGGL((coop<true, 2>), dim3(wgs), dim3(256), 0, sc, d_addr, stages, d_out, stride);
        CK(hipEventRecord(c1, sc));
        if (beside) {
          usleep(300);
          CK(hipEventRecord(s0, ss));
          if (shared)  // one 64 KiB streamer workgroup beside every coop workgroup
            hipLaunchKernelGGL(stream_read, dim3(256), dim3(1024), 64 * 1024, ss, (const u32x4*)d_s, sbytes / 16, 4u,
                               d_out);
          else
            hipLaunchKernelGGL(stream_read, dim3(256 - std::min(wgs, 255u)), dim3(1024), 128 * 1024, ss,
                               (const u32x4*)d_s, sbytes / 16, 4u, d_out);
          CK(hipEventRecord(s1, ss));
        }
        CK(hipDeviceSynchronize());
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, c0, c1));
        if (ms < best) {
          best = ms;
          if (beside) {
            float st = 0.f;
            CK(hipEventElapsedTime(&st, s0, s1));
            sms = st;
          }
        }
      }
      printf("%s%s, %u, %u, %.3f, %.1f, %.1f\n", k.name, beside ? "_beside" : "", S, stages, best,
             bytes / (best * 1e6), beside ? 4.0 * sbytes / (sms * 1e6) : 0.0);
      fflush(stdout);
    }
    CK(hipFree(d_addr));
  }
  // the streamer alone, for its own ceiling
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(s0, ss));
    hipLaunchKernelGGL(stream_read, dim3(128), dim3(1024), 128 * 1024, ss, (const u32x4*)d_s, sbytes / 16, 2u, d_out);
    CK(hipEventRecord(s1, ss));
    CK(hipDeviceSynchronize());
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, s0, s1));
    best = std::min(best, ms);
  }
  printf("streamer_alone_128cu, 0, 0, %.3f, %.1f, 0\n", best, 2.0 * sbytes / (best * 1e6));
  return 0;
}

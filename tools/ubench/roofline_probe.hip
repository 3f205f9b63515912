// Practical ceilings of the two rooflines the path sits under:
//   hbm   read-only streaming of an 8 GiB buffer with global_load_dwordx4
//         (grid-stride, 4 loads in flight per lane), best and median of 10;
//   valu  int32 VALU issue: 8 independent v_add_u32 chains per lane, at 8 waves
//         per SIMD (SIMD-32 pipe saturated) and at 1 wave per SIMD (one wave's
//         own issue cap), reported as lane-ops/s;
//   md5   the K3 step's dependent chain (bitop3 -> add3 -> add -> alignbit -> add)
//         at 1 wave per SIMD, in cycles per step (s_memtime), = the floor of one
//         serial MD5 chain.
// hipcc --offload-arch=gfx950 -O3 -o roofline_probe roofline_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void hbm_read(const u32x4* __restrict__ p, uint64_t n16,
                                                 uint32_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4 a = __builtin_nontemporal_load(p + i);
    const u32x4 b = __builtin_nontemporal_load(p + i + stride);
    const u32x4 c = __builtin_nontemporal_load(p + i + 2 * stride);
    const u32x4 d = __builtin_nontemporal_load(p + i + 3 * stride);
    acc ^= a ^ b ^ c ^ d;
  }
  for (; i < n16; i += stride) acc ^= p[i];
  const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x9e3779b9u) out[0] = r;  // never true on the memset pattern; keeps the loads
}

__global__ __launch_bounds__(256) void hbm_read_plain(const u32x4* __restrict__ p, uint64_t n16,
                                                       uint32_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (; i + 3 * stride < n16; i += 4 * stride) acc ^= p[i] ^ p[i + stride] ^ p[i + 2 * stride] ^ p[i + 3 * stride];
  for (; i < n16; i += stride) acc ^= p[i];
  const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x9e3779b9u) out[0] = r;
}

#define REP8(x) x x x x x x x x
__global__ __launch_bounds__(256) void valu_issue(uint32_t* out, uint32_t iters, uint32_t seed) {
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3u, a2 = a0 ^ 5u, a3 = a0 + 7u, a4 = a0 * 5u,
           a5 = a0 ^ 9u, a6 = a0 + 11u, a7 = a0 * 13u, k = seed | 1u;
  for (uint32_t i = 0; i < iters; i++) {
    REP8(asm volatile(
             "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
             "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
             : "v"(k));)
  }
  const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0x9e3779b9u) out[0] = r;
}

// One MD5 round-1 step per asm block, dependent through b (the K3 critical
// path); 16 steps per iteration.
__global__ __launch_bounds__(64) void md5_chain(uint32_t* out, uint64_t* cyc, uint32_t iters,
                                                uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u, c = seed ^ 0x55u, d = seed + 0x77u, m = seed ^ 0x1234u;
  uint32_t t;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; i++) {
#define MD5STEP(A, B, C, D)                                                           \
  asm volatile(                                                                       \
      "v_add3_u32 %0, %1, %5, %6\n\t"                                                 \
      "v_bitop3_b32 %2, %3, %4, %7 bitop3:0xca\n\t"                                   \
      "v_add_u32 %0, %0, %2\n\t"                                                      \
      "v_alignbit_b32 %0, %0, %0, 25\n\t"                                             \
      "v_add_u32 %1, %0, %3"                                                          \
      : "=&v"(t), "+v"(A), "=&v"(c2)                                                  \
      : "v"(B), "v"(C), "v"(m), "s"(0xd76aa478u), "v"(D));
    uint32_t c2;
    REP8(MD5STEP(a, b, c, d) MD5STEP(d, a, b, c))
#undef MD5STEP
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint32_t r = a ^ b ^ c ^ d ^ t;
  if (r == 0x9e3779b9u) out[0] = r;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <typename F>
static float time_ms(F f, int reps, std::vector<float>& all) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();  // warm-up
  (void)hipDeviceSynchronize();
  for (int r = 0; r < reps; r++) {
    (void)hipEventRecord(e0, 0);
    f();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    all.push_back(ms);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  std::sort(all.begin(), all.end());
  return all[0];
}

int main(int argc, char** argv) {
  const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : 8ull) << 30;
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  u32x4* buf = nullptr;
  uint32_t* out = nullptr;
  uint64_t* cyc = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&cyc, 64));
  CK(hipMemset(buf, 0x5a, bytes));
  CK(hipDeviceSynchronize());
  const uint64_t n16 = bytes / 16;

  printf("{\"device\": \"%s\", \"cus\": %d, \"bytes\": %llu", prop.name, cus, (unsigned long long)bytes);
  for (int variant = 0; variant < 2; variant++) {
    for (int wgs_per_cu : {4, 8, 16}) {
      std::vector<float> all;
      const int grid = cus * wgs_per_cu;
      const float best = time_ms(
          [&] {
            if (variant == 0)
              hbm_read<<<grid, 256>>>(buf, n16, out);
            else
              hbm_read_plain<<<grid, 256>>>(buf, n16, out);
          },
          10, all);
      printf(", \"hbm_%s_wg%d\": {\"best_gbs\": %.1f, \"median_gbs\": %.1f}", variant ? "plain" : "nt",
             wgs_per_cu, bytes / (best * 1e-3) / 1e9, bytes / (all[all.size() / 2] * 1e-3) / 1e9);
    }
  }
  CK(hipGetLastError());

  const uint32_t iters = 4096;
  for (int waves_per_simd : {1, 2, 8}) {
    // 256-thread WG = 4 waves = one per SIMD
    const int grid = cus * waves_per_simd;
    std::vector<float> all;
    const float best = time_ms([&] { valu_issue<<<grid, 256>>>(out, iters, 7u); }, 5, all);
    const double lane_ops = (double)grid * 256 * iters * 64;
    printf(", \"valu_add_%dwps\": {\"best_tops\": %.2f}", waves_per_simd, lane_ops / (best * 1e-3) / 1e12);
  }
  CK(hipGetLastError());

  {
    const uint32_t it2 = 2048;
    std::vector<float> all;
    const int grid = cus * 4;  // 64-thread WGs: one wave per SIMD
    const float best = time_ms([&] { md5_chain<<<grid, 64>>>(out, cyc, it2, 7u); }, 5, all);
    uint64_t c = 0;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    const double steps = (double)it2 * 16;
    printf(", \"md5_step_1wps\": {\"memtime_ticks_per_step\": %.2f, \"ns_per_step\": %.3f, "
           "\"ns_per_block\": %.1f}",
           c / steps, best * 1e6 / steps, best * 1e6 / steps * 64);
  }
  CK(hipGetLastError());
  printf("}\n");
  CK(hipFree(buf));
  return 0;
}

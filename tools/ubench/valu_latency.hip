// Dependent-chain latency (cycles per op) of the VALU ops on the MD5 critical
// path, one wave alone on the chip.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP16(x) x x x x x x x x x x x x x x x x
template <int OP>
__global__ void chain(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3u, c = seed ^ 0x55u;
  uint64_t v64 = ((uint64_t)a << 32) | b;
  __syncthreads();
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    if (OP == 0) { REP16(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));) }
    if (OP == 1) { REP16(asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));) }
    if (OP == 2) { REP16(asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a));) }
    if (OP == 3) { REP16(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xac" : "+v"(a) : "v"(b), "v"(c));) }
    if (OP == 4) { REP16(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));) }
    if (OP == 5) { REP16(asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(v64) : "v"(v64));) }
    if (OP == 6) { REP16(asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a) : "v"(b));) }
    if (OP == 7) {  // md5-like step: bitop3 -> add3 -> alignbit -> add
      REP16(asm volatile("v_bitop3_b32 %1, %0, %2, %3 bitop3:0xac\n\tv_add3_u32 %1, %1, %2, %3\n\tv_alignbit_b32 %1, %1, %1, 25\n\tv_add_u32 %0, %1, %0" : "+v"(a), "=&v"(c) : "v"(b), "v"(seed));)
    }
    if (OP == 8) {  // independent stream (issue rate): 4 independent accumulators
      REP16(asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4" : "+v"(a), "+v"(b), "+v"(c), "+v"(seed) : "v"(seed));)
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a + b + c + (uint32_t)v64;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// waves-per-SIMD scaling of the md5-like chain: blockDim 64/256/512/1024
void scaling(uint32_t* d, uint64_t* c) {
  for (int bd : {64, 256, 512, 1024}) {
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(chain<7>, 1, bd, 0, 0, d, c, 7);
      uint64_t cy = 0; (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("md5 chain, %4d threads (%d waves/SIMD): %6.2f ticks/op per wave\n", bd,
                      bd / 256 ? bd / 256 : 1, (double)cy / (256.0 * 16 * 4));
    }
  }
}

int main() {
  uint32_t* d; uint64_t* c; hipMalloc(&d, 4096); hipMalloc(&c, 64);
  const char* names[] = {"v_add_u32", "v_add3_u32", "v_alignbit_b32", "v_bitop3_b32", "v_xor_b32",
                         "v_lshl_add_u64", "v_lshl_add_u32", "md5 step (4 ops)", "independent add (4 ops)"};
  for (int rep = 0; rep < 2; rep++)
  for (int op = 0; op < 9; op++) {
    switch (op) {
      case 0: hipLaunchKernelGGL(chain<0>, 1, 64, 0, 0, d, c, 7); break;
      case 1: hipLaunchKernelGGL(chain<1>, 1, 64, 0, 0, d, c, 7); break;
      case 2: hipLaunchKernelGGL(chain<2>, 1, 64, 0, 0, d, c, 7); break;
      case 3: hipLaunchKernelGGL(chain<3>, 1, 64, 0, 0, d, c, 7); break;
      case 4: hipLaunchKernelGGL(chain<4>, 1, 64, 0, 0, d, c, 7); break;
      case 5: hipLaunchKernelGGL(chain<5>, 1, 64, 0, 0, d, c, 7); break;
      case 6: hipLaunchKernelGGL(chain<6>, 1, 64, 0, 0, d, c, 7); break;
      case 7: hipLaunchKernelGGL(chain<7>, 1, 64, 0, 0, d, c, 7); break;
      case 8: hipLaunchKernelGGL(chain<8>, 1, 64, 0, 0, d, c, 7); break;
    }
    uint64_t cy = 0; hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    double per = (double)cy / (256.0 * 16 * ((op >= 7) ? 4 : 1));
    if (rep) printf("%-26s %6.2f cycles/op (s_memtime ticks)\n", names[op], per);
  }
  scaling(d, c);
  return 0;
}

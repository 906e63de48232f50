// Microbenchmark: issue cost of the instructions in the noise path on gfx950.
// One wave per SIMD (256 blocks x 256 threads), 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint32_t seed, long long iters) {
  uint32_t a[8];
  double d[8];
  for (int j = 0; j < 8; ++j) { a[j] = seed * (threadIdx.x + j + 1); d[j] = 1.0 + 1e-9 * (a[j] & 1023); }
  const uint64_t t0 = __builtin_readcyclecounter();
  for (long long it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) { uint64_t p = (uint64_t)0xD2511F53u * a[j]; a[j] = (uint32_t)(p >> 32) ^ (uint32_t)p; }
      if (OP == 1) d[j] = fma(d[j], 1.0000001, 1e-12);
      if (OP == 2) a[j] = (a[j] ^ 0x9E3779B9u) + (a[j] >> 3);
      if (OP == 3) { a[j] = __umulhi(a[j], 0xCD9E8D57u) ^ (a[j] * 0xCD9E8D57u); }
      if (OP == 4) d[j] = d[j] * 1.0000001 + d[j];
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  double acc = 0; uint32_t x = 0;
  for (int j = 0; j < 8; ++j) { acc += d[j]; x ^= a[j]; }
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 123.0 && x == 7u) out[0] = 0;
}

int main() {
  uint64_t* d; hipMalloc(&d, 1024 * 8);
  const long long iters = 20000;
  const char* names[] = {"mad_u64_u32 + xor", "fma_f64", "xor+shr+add (3x 32-bit)", "mul_hi+mul_lo+xor", "mul_f64+add_f64"};
  for (int op = 0; op < 5; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, d, 7u, iters); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, d, 7u, iters); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, d, 7u, iters); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, d, 7u, iters); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, d, 7u, iters); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      uint64_t h[4]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      // 4 waves per CU = 1 wave per SIMD; per wave 8*iters ops
      const double ops_per_simd = 8.0 * iters;
      if (rep) printf("%-28s %.2f ns/op-per-SIMD  (%.2f cycles @2.4GHz) counter %.2f cyc/op\n", names[op],
                      ms * 1e6 / ops_per_simd, ms * 1e6 / ops_per_simd * 2.4, (double)h[1] / ops_per_simd);
    }
  }
  return 0;
}

// Issue cost of the instructions on the noise path: per-wave cycles of
// v_mad_u64_u32 (Philox's 32 x 32 -> 64 multiply), v_bitop3_b32, v_fma_f64,
// v_mul_lo_u32 and of one whole Philox4x32-10 block, from long chains of
// independent operations (8 per lane) over a grid that fills every SIMD.
//   hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#include "../../viabel_amd/csrc/vb_device.hpp"

constexpr int ITER = 256, CH = 8;

__global__ void k_mad(uint32_t* out, uint32_t s) {
  uint32_t x[CH];
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const uint64_t p = (uint64_t)0xD2511F53u * x[c];
      x[c] = (uint32_t)(p >> 32) ^ (uint32_t)p;
    }
  uint32_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= x[c];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_mullo(uint32_t* out, uint32_t s) {
  uint32_t x[CH];
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = x[c] * 0xD2511F53u + s;
  uint32_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= x[c];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_bitop3(uint32_t* out, uint32_t s) {
  uint32_t x[CH];
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = __builtin_amdgcn_bitop3_b32(x[c], x[(c + 1) % CH], s, 0x96);
  uint32_t r = 0;
  for (int c = 0; c < CH; ++c) r ^= x[c];
  if (r == 0x12345) out[0] = r;
}
__global__ void k_fma(uint32_t* out, uint32_t s) {
  double x[CH];
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x + c * (double)s;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = vbd::hfma(x[c], 0.999999, 1e-7);
  double r = 0;
  for (int c = 0; c < CH; ++c) r += x[c];
  if (r == 0.125) out[0] = 1;
}
__global__ void k_philox(uint32_t* out, uint32_t s) {
  uint32_t r = 0;
  for (int i = 0; i < ITER / 8; ++i) {
    const vbd::u4 w = vbd::philox(threadIdx.x, i, blockIdx.x, 7, s, s + 1);
    r ^= w.x ^ w.y ^ w.z ^ w.w;
  }
  if (r == 0x12345) out[0] = r;
}

int main() {
  uint32_t* out;
  (void)hipMalloc(&out, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipDeviceProp_t pr;
  (void)hipGetDeviceProperties(&pr, 0);
  const int cus = pr.multiProcessorCount;
  const double ghz = pr.clockRate * 1e-6;
  // 8 waves per SIMD: 4 SIMDs x 8 = 32 waves per CU = 8 blocks of 256
  const int blocks = cus * 8, threads = 256;
  const double waves_per_simd = (double)blocks * threads / 64 / (cus * 4);
  struct K { const char* name; void (*f)(uint32_t*, uint32_t); double ops; };
  K ks[] = {{"v_mad_u64_u32 (+1 xor)", k_mad, (double)ITER * CH},
            {"v_mul_lo_u32 + add", k_mullo, (double)ITER * CH},
            {"v_bitop3_b32", k_bitop3, (double)ITER * CH},
            {"v_fma_f64", k_fma, (double)ITER * CH},
            {"philox4x32-10 block", k_philox, (double)ITER / 8}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 3u);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2)
        printf("%-26s %8.3f ms  %7.2f SIMD cycles per wave-op (at %.2f GHz nominal)\n", k.name, ms,
               ms * 1e-3 * ghz * 1e9 / (waves_per_simd * k.ops), ghz);
    }
  }
  return 0;
}

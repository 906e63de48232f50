// vb_probe.hip — peak-rate microbenchmarks (measurement support for bench.py's
// roofline fractions; BASELINE.md §2: "both peaks must be confirmed with
// microbenchmarks on the box").  No reference counterpart.
//
//   kind 0  HBM copy     nontemporal 16-byte loads + stores over two buffers far
//                        past the 256 MB Infinity Cache, one slab per 1024-thread
//                        block; GB/s of read + written bytes
//   kind 1  HBM read     nontemporal 16-byte loads, one slab per block, folded into
//                        one XOR per thread; GB/s read
//   kind 2  fp64 MFMA    v_mfma_f64_16x16x4_f64, 4 independent accumulators per
//                        wave, 4 waves per SIMD; TFLOP/s
//   kind 3  fp64 VALU    v_fma_f64, 8 independent chains per lane, 4 waves per
//                        SIMD; G wave-instructions/s (the VALU issue peak the
//                        fp64 kernels are priced against)
//   kind 4  u64 multiply v_mad_u64_u32 chains (Philox's multiply), as kind 3
#include "../../include/viabel_amd.h"
#include "vb_internal.hpp"

#include <hip/hip_runtime.h>

namespace vbk {
namespace {

using u4 = unsigned __attribute__((ext_vector_type(4)));
using d4 = double __attribute__((ext_vector_type(4)));

// copy: each 1024-thread block (one per CU) streams one contiguous slab with
// nontemporal loads and stores, 4 vectors in flight per thread -- the fastest
// copy form of the round-5 sweep (scripts/ubench/hbm_probe2.hip,
// profiles/r05/hbm_probe2.log: 5.71-5.73 TB/s against 5.31-5.45 for 256-thread
// slabs with plain loads / stores, 4.99 for hipMemcpy device-to-device; round 4's
// grid-stride forms 4.2-5.2, profiles/r04/hbm_probe_variants.log).  Still below
// the 6.29 TB/s float4 copy of MI355X_MICROARCH.md, so bench.py reports the
// fractions against that figure as well.
__global__ __launch_bounds__(1024) void probe_copy_kernel(const u4* __restrict__ src,
                                                          u4* __restrict__ dst, long long n) {
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  long long i = b0 + threadIdx.x;
  for (; i + 3 * 1024 < b1; i += 4 * 1024) {
    const u4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + 1024),
             c = __builtin_nontemporal_load(src + i + 2048), d = __builtin_nontemporal_load(src + i + 3072);
    __builtin_nontemporal_store(a, dst + i);
    __builtin_nontemporal_store(b, dst + i + 1024);
    __builtin_nontemporal_store(c, dst + i + 2048);
    __builtin_nontemporal_store(d, dst + i + 3072);
  }
  for (; i < b1; i += 1024) dst[i] = src[i];
}

// read: each 256-thread block (two per CU) streams one slab with nontemporal
// 16-byte loads, 8 in flight per thread, folded into one XOR per thread: 6.7-7.1
// TB/s in the round-5 sweep (the grid-stride form of round 4: 5.5-6.0)
__global__ __launch_bounds__(256) void probe_read_kernel(const u4* __restrict__ src, long long n,
                                                         unsigned* __restrict__ out) {
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
  long long i = b0 + threadIdx.x;
  u4 acc = {0u, 0u, 0u, 0u};
  for (; i + 7 * 256 < b1; i += 8 * 256) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= __builtin_nontemporal_load(src + i + u * 256);
  }
  for (; i < b1; i += 256) acc ^= src[i];
  out[(long long)blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

__global__ __launch_bounds__(256) void probe_mfma_kernel(double* out, int iters) {
  d4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = d4{0, 0, 0, 0};
  const double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void probe_fma_kernel(double* out, int iters) {
  double x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3 + j;
  const double m = 0.999999, c = 1e-7 * blockIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fma(x[j], m, c);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void probe_mad64_kernel(double* out, int iters) {
  unsigned long long x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + 977u * j;
  const unsigned m = 0xD2511F53u + blockIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (unsigned long long)m * (unsigned)x[j] + (x[j] >> 32);
  }
  unsigned long long s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= x[j];
  out[blockIdx.x * 256 + threadIdx.x] = (double)(s & 0xFFFF);
}

}  // namespace

// rate of one probe (see the file header), best of `reps` timed launches after
// one untimed launch; buffers are allocated and freed here
int probe_rate(int kind, long long n, int reps, hipStream_t st, double* out) {
  if (kind < 0 || kind > 4) return vb_set_error(-1, "vb_peak_probe: kind in [0, 4]");
  if (reps < 1 || n < 1) return vb_set_error(-1, "vb_peak_probe: n >= 1, reps >= 1");
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  void *a = nullptr, *b = nullptr;
  const long long nv = kind <= 1 ? n / 16 : 0;        // 16-byte vectors
  const unsigned blocks = kind == 0 ? (unsigned)ncu : kind == 1 ? (unsigned)ncu * 2 : (unsigned)ncu * 4;
  const size_t abytes = kind <= 1 ? (size_t)nv * 16 : 0;
  const size_t bbytes = kind == 0 ? abytes : sizeof(double) * blocks * 256;
  if (abytes && hipMalloc(&a, abytes) != hipSuccess) {
    (void)hipGetLastError();
    return vb_set_error(-3, "vb_peak_probe: hipMalloc(%zu) failed", abytes);
  }
  if (hipMalloc(&b, bbytes) != hipSuccess) {
    (void)hipGetLastError();
    if (a) (void)hipFree(a);
    return vb_set_error(-3, "vb_peak_probe: hipMalloc(%zu) failed", bbytes);
  }
  if (a) (void)hipMemsetAsync(a, 1, abytes, st);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = (int)std::min<long long>(n, 1 << 30);
  auto launch = [&]() {
    switch (kind) {
      case 0:
        hipLaunchKernelGGL(probe_copy_kernel, dim3(blocks), dim3(1024), 0, st, (const u4*)a, (u4*)b, nv);
        break;
      case 1:
        hipLaunchKernelGGL(probe_read_kernel, dim3(blocks), dim3(256), 0, st, (const u4*)a, nv,
                           (unsigned*)b);
        break;
      case 2: hipLaunchKernelGGL(probe_mfma_kernel, dim3(blocks), dim3(256), 0, st, (double*)b, iters); break;
      case 3: hipLaunchKernelGGL(probe_fma_kernel, dim3(blocks), dim3(256), 0, st, (double*)b, iters); break;
      default: hipLaunchKernelGGL(probe_mad64_kernel, dim3(blocks), dim3(256), 0, st, (double*)b, iters); break;
    }
  };
  launch();
  float best = 0.f;
  int rc = 0;
  for (int r = 0; r < reps && !rc; ++r) {
    (void)hipEventRecord(e0, st);
    launch();
    (void)hipEventRecord(e1, st);
    if (hipEventSynchronize(e1) != hipSuccess) {
      rc = vb_set_error(-2, "vb_peak_probe: kernel failed: %s", hipGetErrorString(hipGetLastError()));
      break;
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r == 0 || ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (a) (void)hipFree(a);
  (void)hipFree(b);
  if (rc) return rc;
  const double sec = best * 1e-3;
  const double waves = (double)blocks * 4;          // 256-thread blocks
  switch (kind) {
    case 0: *out = 2.0 * (double)nv * 16 / sec / 1e9; break;
    case 1: *out = (double)nv * 16 / sec / 1e9; break;
    case 2: *out = 2.0 * 16 * 16 * 4 * 4.0 * iters * waves / sec / 1e12; break;
    default: *out = 8.0 * iters * waves / sec / 1e9; break;   // wave-instructions
  }
  return 0;
}

}  // namespace vbk

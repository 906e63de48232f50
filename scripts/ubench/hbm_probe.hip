// HBM copy / read variants for vb_probe.hip's peak probe: which form of a
// streaming kernel reaches the chip's copy peak.
//   hipcc --offload-arch=gfx950 -O3 hbm_probe.hip -o hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>

using u4 = unsigned __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const u4* __restrict__ src, u4* __restrict__ dst,
                                              long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// contiguous chunk per block (each block streams its own slab)
template <int U>
__global__ __launch_bounds__(256) void copy_slab(const u4* __restrict__ src, u4* __restrict__ dst,
                                                 long long n) {
  const long long per = n / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per;
  for (long long i = b0 + threadIdx.x; i + (U - 1) * 256 < b0 + per; i += U * 256) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * 256] = v[u];
  }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_k(const u4* __restrict__ src, long long n, unsigned* out) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  u4 acc = {0u, 0u, 0u, 0u};
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <class F>
float best_ms(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  float best = 1e9f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a, 0);
    f();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const long long bytes = 1ll << 30, n = bytes / 16;
  u4 *a, *b;
  unsigned* o;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMalloc(&o, 256 * 1024 * 64 * 4);
  hipMemset(a, 1, bytes);
  hipMemset(b, 2, bytes);
  for (int bpc : {4, 8, 16, 32}) {
    const int g = 256 * bpc;
    float t;
    t = best_ms([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, 8);
    printf("copy   u4 blocks/CU %2d: %7.1f GB/s\n", bpc, 2.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((copy_k<8, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, 8);
    printf("copy   u8 blocks/CU %2d: %7.1f GB/s\n", bpc, 2.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, 8);
    printf("copy nt u4 blocks/CU %2d: %7.1f GB/s\n", bpc, 2.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((copy_slab<4>), dim3(g), dim3(256), 0, 0, a, b, n); }, 8);
    printf("slab   u4 blocks/CU %2d: %7.1f GB/s\n", bpc, 2.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((read_k<4, false>), dim3(g), dim3(256), 0, 0, a, n, o); }, 8);
    printf("read   u4 blocks/CU %2d: %7.1f GB/s\n", bpc, 1.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((read_k<8, true>), dim3(g), dim3(256), 0, 0, a, n, o); }, 8);
    printf("read nt u8 blocks/CU %2d: %7.1f GB/s\n", bpc, 1.0 * bytes / t / 1e6);
  }
  return 0;
}

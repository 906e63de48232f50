// More HBM copy / read forms for vb_probe.hip's peak probe (round 5): slabs with
// nontemporal loads / stores, deeper unrolls, bigger blocks, and the runtime's
// own device-to-device copy, on 1 GiB buffers (4x the Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 hbm_probe2.hip -o hbm_probe2
#include <hip/hip_runtime.h>

#include <cstdio>

using u4 = unsigned __attribute__((ext_vector_type(4)));

// each block streams one contiguous slab; NTL / NTS: nontemporal loads / stores
template <int U, bool NTL, bool NTS, int NT>
__global__ __launch_bounds__(NT) void slab(const u4* __restrict__ src, u4* __restrict__ dst, long long n) {
  const long long per = n / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per;
  for (long long i = b0 + threadIdx.x; i + (U - 1) * NT < b0 + per; i += U * NT) {
    u4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(src + i + u * NT) : src[i + u * NT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], dst + i + u * NT);
      else dst[i + u * NT] = v[u];
    }
  }
}

template <int U, bool NTL, int NT>
__global__ __launch_bounds__(NT) void slab_read(const u4* __restrict__ src, long long n, unsigned* out) {
  const long long per = n / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per;
  u4 acc = {0u, 0u, 0u, 0u};
  for (long long i = b0 + threadIdx.x; i + (U - 1) * NT < b0 + per; i += U * NT) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= NTL ? __builtin_nontemporal_load(src + i + u * NT) : src[i + u * NT];
  }
  out[blockIdx.x * NT + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
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
  (void)hipMalloc(&a, bytes);
  (void)hipMalloc(&b, bytes);
  (void)hipMalloc(&o, 256 * 64 * 1024 * 4);
  (void)hipMemset(a, 1, bytes);
  (void)hipMemset(b, 2, bytes);
  float t = best_ms([&] { (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }, 8);
  printf("hipMemcpy D2D            : %7.1f GB/s\n", 2.0 * bytes / t / 1e6);
  for (int bpc : {2, 4, 8, 16}) {
    const int g = 256 * bpc;
#define RUN(NAME, ...)                                                                          \
    t = best_ms([&] { hipLaunchKernelGGL((__VA_ARGS__), dim3(g), dim3(256), 0, 0, a, b, n); }, 8); \
    printf("%-24s bpc %2d: %7.1f GB/s\n", NAME, bpc, 2.0 * bytes / t / 1e6);
    RUN("slab u4", slab<4, false, false, 256>)
    RUN("slab u8", slab<8, false, false, 256>)
    RUN("slab u4 nt-load", slab<4, true, false, 256>)
    RUN("slab u4 nt-store", slab<4, false, true, 256>)
    RUN("slab u4 nt-both", slab<4, true, true, 256>)
    RUN("slab u8 nt-both", slab<8, true, true, 256>)
#undef RUN
    t = best_ms([&] { hipLaunchKernelGGL((slab_read<8, true, 256>), dim3(g), dim3(256), 0, 0, a, n, o); }, 8);
    printf("%-24s bpc %2d: %7.1f GB/s\n", "read slab u8 nt", bpc, 1.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((slab_read<8, false, 256>), dim3(g), dim3(256), 0, 0, a, n, o); }, 8);
    printf("%-24s bpc %2d: %7.1f GB/s\n", "read slab u8", bpc, 1.0 * bytes / t / 1e6);
  }
  for (int bpc : {1, 2, 4}) {
    const int g = 256 * bpc;
    t = best_ms([&] { hipLaunchKernelGGL((slab<4, true, true, 1024>), dim3(g), dim3(1024), 0, 0, a, b, n); }, 8);
    printf("%-24s bpc %2d: %7.1f GB/s\n", "slab1024 u4 nt-both", bpc, 2.0 * bytes / t / 1e6);
    t = best_ms([&] { hipLaunchKernelGGL((slab<4, false, false, 1024>), dim3(g), dim3(1024), 0, 0, a, b, n); }, 8);
    printf("%-24s bpc %2d: %7.1f GB/s\n", "slab1024 u4", bpc, 2.0 * bytes / t / 1e6);
  }
  return 0;
}

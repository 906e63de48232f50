// Peak rate of v_mfma_f64_16x16x4_f64: back-to-back issue with independent
// accumulators, all CUs.  hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.cpp -o mfma_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
using d4 = double __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k(double* out, int iters) {
  d4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 + blockIdx.x * 1e-6;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  double* o;
  hipMalloc(&o, 256 * 4096 * 8);
  const int iters = 20000;
  for (int wpb : {1, 2, 4}) {
    for (int blocks : {256, 1024}) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64 * wpb), 0, 0, o, 100);
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64 * wpb), 0, 0, o, iters);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double fl = 2.0 * 16 * 16 * 4 * 4.0 * iters * blocks * wpb;
      printf("waves/block %d blocks %d: %.2f ms  %.1f TF/s  cycles/MFMA/wave-on-SIMD (at 2.4GHz, waves per SIMD %.2f): %.1f\n",
             wpb, blocks, ms, fl / (ms * 1e-3) / 1e12, blocks * wpb / 1024.0,
             ms * 1e-3 * 2.4e9 / (4.0 * iters) / (blocks * wpb / 1024.0 > 1 ? blocks * wpb / 1024.0 : 1));
    }
  }
  return 0;
}

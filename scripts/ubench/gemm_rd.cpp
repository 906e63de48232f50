// Register-direct small-tile fp64 GEMM probe (round 6, config 4): each block owns a
// 16 x 16 output tile (or 32 x 16) and 4 waves split K in four; every lane loads
// all of its MFMA operands for its k quarter straight into registers (no LDS
// staging: all loads in flight at once), runs its MFMA chains, and the 4 k parts
// are summed through LDS.  Compared with the production 32 x 32 LDS-DMA kernel
// (vbk::gemm) on cold operands (8 rotating operand sets), for the config-4 shapes:
// 512^3 (full), 128 x 512 x 512 (the N-row products x = z S and the target).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_rd.cpp -o gemm_rd
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using d4 = double __attribute__((ext_vector_type(4)));

// TR = 16 * RT rows per block (RT row sub-tiles of 16), 16 columns, K = 16 KL.
// Step s of wave w, lane quad kq uses k = w K/4 + kq KL/4... (see below).
template <int KL, int RT>
__global__ __launch_bounds__(256) void gemm_rd(const double* __restrict__ A,
                                               const double* __restrict__ B, double* C, int lda,
                                               int ldb, int ldc) {
  constexpr int KQ = KL / 4;   // k per lane quad per wave (contiguous)
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int r = l & 15, kq = l >> 4;
  const int i0 = blockIdx.y * 16 * RT, j0 = blockIdx.x * 16;
  const int kb = w * KL + kq * KQ;   // this lane's first k
  double av[RT][KQ], bv[KQ];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const double* a = A + (long long)(i0 + 16 * rt + r) * lda + kb;
#pragma unroll
    for (int s = 0; s < KQ; ++s) av[rt][s] = a[s];
  }
  const double* b = B + (long long)kb * ldb + j0 + r;
#pragma unroll
  for (int s = 0; s < KQ; ++s) bv[s] = b[(long long)s * ldb];
  d4 acc[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[rt][c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < KQ; ++s)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      acc[rt][s & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[rt][s], bv[s], acc[rt][s & 3], 0, 0, 0);
  __shared__ double red[3][RT][4][64];
  d4 r4[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) r4[rt] = (acc[rt][0] + acc[rt][1]) + (acc[rt][2] + acc[rt][3]);
  if (w > 0) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w - 1][rt][i][l] = r4[rt][i];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double v = r4[rt][i] + red[0][rt][i][l] + red[1][rt][i][l] + red[2][rt][i][l];
        C[(long long)(i0 + 16 * rt + kq + 4 * i) * ldc + j0 + r] = v;
      }
  }
}

int main(int argc, char** argv) {
  const int NSET = 8, reps = 400;
  const int D = 512;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  const size_t dd = (size_t)D * D;
  std::vector<double> h(dd);
  double *A[NSET], *B[NSET], *C[NSET];
  for (int s = 0; s < NSET; ++s)
    for (double** p : {&A[s], &B[s], &C[s]}) {
      CK(hipMalloc(p, dd * 8));
      for (auto& x : h) x = nd(rng);
      CK(hipMemcpy(*p, h.data(), dd * 8, hipMemcpyHostToDevice));
    }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto timeit = [&](const char* name, int M, auto&& launch) {
    for (int r = 0; r < 50; ++r) launch(r % NSET);
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) launch(r % NSET);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-28s M=%4d %7.2f us/launch %6.1f TF/s\n", name, M, us,
           2.0 * M * (double)D * D / (us * 1e-6) / 1e12);
  };
  // correctness vs the production kernel
  auto check = [&](int M, auto&& launch) -> double {
    vbk::GemmOp g{};
    g.M = M; g.N = D; g.K = D; g.A = A[0]; g.lda = D; g.B = B[0]; g.ldb = D; g.C = C[1]; g.ldc = D;
    g.alpha = 1.0;
    vbk::gemm(g, 0);
    launch(0);
    hipDeviceSynchronize();
    std::vector<double> x((size_t)M * D), y((size_t)M * D);
    hipMemcpy(x.data(), C[0], x.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(y.data(), C[1], y.size() * 8, hipMemcpyDeviceToHost);
    double e = 0;
    for (size_t i = 0; i < x.size(); ++i) e = fmax(e, fabs(x[i] - y[i]) / (1 + fabs(y[i])));
    return e;
  };
  for (int M : {512, 128}) {
    auto prod = [&](int s) {
      vbk::GemmOp g{};
      g.M = M; g.N = D; g.K = D; g.A = A[s]; g.lda = D; g.B = B[s]; g.ldb = D; g.C = C[s]; g.ldc = D;
      g.alpha = 1.0;
      vbk::gemm(g, 0);
    };
    timeit("production 32x32 LDS-DMA", M, prod);
    auto rd16 = [&](int s) {
      hipLaunchKernelGGL((gemm_rd<128, 1>), dim3(D / 16, M / 16), dim3(256), 0, 0, A[s], B[s],
                         C[s == 0 ? 0 : s], D, D, D);
    };
    printf("  rd 16x16 err vs production %.2e\n", check(M, rd16));
    timeit("register-direct 16x16", M, rd16);
    auto rd32 = [&](int s) {
      hipLaunchKernelGGL((gemm_rd<128, 2>), dim3(D / 16, M / 32), dim3(256), 0, 0, A[s], B[s],
                         C[s == 0 ? 0 : s], D, D, D);
    };
    printf("  rd 32x16 err vs production %.2e\n", check(M, rd32));
    timeit("register-direct 32x16", M, rd32);
  }
  return 0;
}

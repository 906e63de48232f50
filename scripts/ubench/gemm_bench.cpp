// fp64 GEMM microbenchmark: vbk::gemm (vb_gemm.hpp) against rocblas_dgemm on the
// full-rank path's shapes.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_bench.cpp -o gemm_bench -lrocblas
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  struct Case { int M, N, K; bool ta, tb; bool ks; };
#ifdef SPLITK_PROBE
  Case cases[] = {{512, 512, 512, false, false, false}, {512, 512, 256, false, false, false},
                  {1024, 512, 256, false, false, false}, {512, 512, 128, false, false, false},
                  {2048, 512, 128, false, false, false}, {1024, 1024, 256, false, false, false}};
#else
  Case cases[] = {{512, 512, 512, false, false, false}, {512, 512, 512, false, true, false},
                  {512, 512, 512, true, false, false},  {128, 512, 512, false, false, false},
                  {512, 512, 128, true, false, true},   {1024, 1024, 1024, false, false, false},
                  {37, 45, 29, true, true, true}};
#endif
  rocblas_handle h;
  rocblas_create_handle(&h);
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  for (const Case& c : cases) {
    const size_t na = (size_t)c.M * c.K, nb = (size_t)c.K * c.N, nc = (size_t)c.M * c.N;
    std::vector<double> A(na), B(nb), ks(c.K), C(nc), R(nc);
    for (auto& x : A) x = nd(rng);
    for (auto& x : B) x = nd(rng);
    for (auto& x : ks) x = nd(rng);
    double *dA, *dB, *dC, *dR, *dK, *dAs;
    CK(hipMalloc(&dA, na * 8)); CK(hipMalloc(&dB, nb * 8)); CK(hipMalloc(&dC, nc * 8));
    CK(hipMalloc(&dR, nc * 8)); CK(hipMalloc(&dK, c.K * 8)); CK(hipMalloc(&dAs, na * 8));
    CK(hipMemcpy(dA, A.data(), na * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), nb * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dK, ks.data(), c.K * 8, hipMemcpyHostToDevice));
    // reference: scale A's k entries on the host when ks
    std::vector<double> As = A;
    if (c.ks)
      for (int i = 0; i < c.M; ++i)
        for (int k = 0; k < c.K; ++k) (c.ta ? As[(size_t)k * c.M + i] : As[(size_t)i * c.K + k]) *= ks[k];
    CK(hipMemcpy(dAs, As.data(), na * 8, hipMemcpyHostToDevice));
    vbk::GemmOp g{};
    g.ta = c.ta; g.tb = c.tb; g.M = c.M; g.N = c.N; g.K = c.K;
    g.A = dA; g.lda = c.ta ? c.M : c.K; g.B = dB; g.ldb = c.tb ? c.K : c.N;
    g.C = dC; g.ldc = c.N; g.alpha = 1.0; g.beta = 0.0; g.kscale = c.ks ? dK : nullptr;
    // rocBLAS is column-major: C^T = op(B)^T op(A)^T
    const double one = 1.0, zero = 0.0;
    auto rb = [&]() {
      return rocblas_dgemm(h, c.tb ? rocblas_operation_transpose : rocblas_operation_none,
                           c.ta ? rocblas_operation_transpose : rocblas_operation_none, c.N, c.M,
                           c.K, &one, dB, (int)g.ldb, dAs, (int)g.lda, &zero, dR, c.N);
    };
    rb();
    CK(vbk::gemm(g, 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(C.data(), dC, nc * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(R.data(), dR, nc * 8, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (size_t i = 0; i < nc; ++i) { err = fmax(err, fabs(C[i] - R[i])); mx = fmax(mx, fabs(R[i])); }
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int reps = 200;
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) vbk::gemm(g, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms_v; hipEventElapsedTime(&ms_v, e0, e1);
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) rb();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms_r; hipEventElapsedTime(&ms_r, e0, e1);
    const double fl = 2.0 * c.M * c.N * c.K;
    printf("M=%4d N=%4d K=%4d ta=%d tb=%d ks=%d  vbk %7.2f us (%5.1f TF/s)  rocblas %7.2f us (%5.1f TF/s)  max|err|/max %.2e\n",
           c.M, c.N, c.K, c.ta, c.tb, c.ks, ms_v * 1e3 / reps, fl / (ms_v * 1e-3 / reps) / 1e12,
           ms_r * 1e3 / reps, fl / (ms_r * 1e-3 / reps) / 1e12, err / mx);
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dR); hipFree(dK); hipFree(dAs);
  }
  rocblas_destroy_handle(h);
  return 0;
}

// Symmetric-sum product V = A X + X A (vb_symsum.hpp, 256 blocks of 16 x 32 x 2D
// work at D = 512) against the plain D^3 product C = A X (vb_gemm.hpp) on cold
// operands: NSET (A, X, C) sets cycled on one stream.  Checks V against a host
// product.   hipcc --offload-arch=gfx950 -O3 -std=c++17 symsum_bench.cpp -o symsum_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_symsum.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 512;
  const int NSET = 8, reps = 200;
  const size_t dd = (size_t)D * D;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::vector<double> h(dd);
  double *A[NSET], *X[NSET], *C[NSET];
  for (int s = 0; s < NSET; ++s) {
    for (double** p : {&A[s], &X[s], &C[s]}) {
      CK(hipMalloc(p, dd * 8));
      for (int i = 0; i < D; ++i)
        for (int j = 0; j <= i; ++j) h[(size_t)i * D + j] = h[(size_t)j * D + i] = nd(rng);
      CK(hipMemcpy(*p, h.data(), dd * 8, hipMemcpyHostToDevice));
    }
  }
  const int kt = argc > 2 ? atoi(argv[2]) : 0;
  CK(vbk::symsum::plain(A[0], X[0], D, 1.0, C[0], 0, kt));
  CK(hipDeviceSynchronize());
  std::vector<double> a(dd), x(dd), c(dd);
  CK(hipMemcpy(a.data(), A[0], dd * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(x.data(), X[0], dd * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), C[0], dd * 8, hipMemcpyDeviceToHost));
  double err = 0.0, asym = 0.0;
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) {
      double r = 0.0;
      for (int k = 0; k < D; ++k) r += a[(size_t)i * D + k] * x[(size_t)k * D + j] + x[(size_t)i * D + k] * a[(size_t)k * D + j];
      err = fmax(err, fabs(r - c[(size_t)i * D + j]) / (1.0 + fabs(r)));
      asym = fmax(asym, fabs(c[(size_t)i * D + j] - c[(size_t)j * D + i]));
    }
  printf("symsum D=%d kt=%d gs=%d max rel err %.3e, max |V - V^T| %.3e\n", D, kt, VB_SS_GS, err, asym);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 2; ++mode) {
    for (int pass = 0; pass < 2; ++pass) {
      hipEventRecord(e0, 0);
      for (int r = 0; r < reps; ++r) {
        const int s = r % NSET;
        if (mode == 0) {
          vbk::GemmOp g{};
          g.M = g.N = g.K = D;
          g.A = A[s]; g.lda = D; g.B = X[s]; g.ldb = D; g.C = C[s]; g.ldc = D;
          g.alpha = 1.0;
          CK(vbk::gemm(g, 0));
        } else {
          CK(vbk::symsum::plain(A[s], X[s], D, 1.0, C[s], 0, kt));
        }
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (pass) printf("%s: %.2f us per launch\n", mode ? "symsum A X + X A" : "plain gemm A X", 1e3 * ms / reps);
    }
  }
  return 0;
}

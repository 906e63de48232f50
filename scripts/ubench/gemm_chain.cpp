// Cold-operand fp64 GEMM chain: the full-rank step's 512^3 products read operands
// the previous kernel just wrote, not L2-hot ones.  This bench cycles through
// NSET independent (A, B, C) sets (NSET x 6 MB > one XCD's 4 MB L2) on one
// stream and reports the mean time per product.  Build twice to compare tile
// placements:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_chain.cpp -o gemm_chain
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVB_GEMM_NO_XCD gemm_chain.cpp -o gemm_chain_id
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 512;
  const int NSET = 8, reps = 400;
  const size_t dd = (size_t)D * D;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::vector<double> h(dd);
  double *A[NSET], *B[NSET], *C[NSET];
  for (int s = 0; s < NSET; ++s) {
    for (double** p : {&A[s], &B[s], &C[s]}) {
      CK(hipMalloc(p, dd * 8));
      for (auto& x : h) x = nd(rng);
      CK(hipMemcpy(*p, h.data(), dd * 8, hipMemcpyHostToDevice));
    }
  }
  auto op = [&](int s, bool dual) {
    vbk::GemmOp g{};
    g.M = g.N = g.K = D;
    g.A = A[s]; g.lda = D; g.B = B[s]; g.ldb = D; g.C = C[s]; g.ldc = D;
    g.alpha = 1.0;
    if (dual) { g.A2 = B[s]; g.B2 = A[s]; g.alpha2 = 1.0; }
    return g;
  };
  // correctness of one product against a host reference (first rows)
  CK(vbk::gemm(op(0, false), 0));
  CK(hipDeviceSynchronize());
  std::vector<double> a(dd), b(dd), c(dd);
  CK(hipMemcpy(a.data(), A[0], dd * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), B[0], dd * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), C[0], dd * 8, hipMemcpyDeviceToHost));
  double err = 0.0;
  for (int i = 0; i < D; i += 37)
    for (int j = 0; j < D; ++j) {
      double r = 0.0;
      for (int k = 0; k < D; ++k) r += a[(size_t)i * D + k] * b[(size_t)k * D + j];
      err = fmax(err, fabs(r - c[(size_t)i * D + j]) / (1.0 + fabs(r)));
    }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int only = argc > 2 ? atoi(argv[2]) : -1;   // run one mode (0 single, 1 dual, 2 group2)
  for (int mode = 0; mode < 3; ++mode) {
    if (only >= 0 && mode != only) continue;
    for (int r = 0; r < 50; ++r) {
      if (mode == 2) {
        vbk::GemmOp g2[2] = {op(r % NSET, false), op((r + 1) % NSET, false)};
        vbk::gemm_group(g2, 2, 0);
      } else {
        vbk::gemm(op(r % NSET, mode == 1), 0);
      }
    }
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) {
      if (mode == 2) {
        vbk::GemmOp g2[2] = {op(r % NSET, false), op((r + 3) % NSET, false)};
        vbk::gemm_group(g2, 2, 0);
      } else {
        vbk::gemm(op(r % NSET, mode == 1), 0);
      }
    }
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double fl = 2.0 * D * (double)D * D * (mode == 0 ? 1 : 2);
    printf("D=%d %-7s %7.2f us/launch  %5.1f TF/s  (host-check rel err %.1e)\n", D,
           mode == 0 ? "single" : mode == 1 ? "dual" : "group2", us, fl / (us * 1e-6) / 1e12, err);
  }
  return 0;
}

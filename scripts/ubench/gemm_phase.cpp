// Phase timing of the fp64 LDS-DMA GEMM (vb_gemm.hpp built with VB_GEMM_PROF):
// a 512^3 product on cold operands (8 buffer sets cycled), then the per-phase
// timestamps of every block of the last launch -- where a launch's time goes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DVB_GEMM_PROF gemm_phase.cpp -o gemm_phase
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int D = 512, NSET = 8;
  const int sym = argc > 1 ? atoi(argv[1]) : 0;
  const size_t dd = (size_t)D * D;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::vector<double> h(dd);
  double *A[NSET], *B[NSET], *C[NSET];
  for (int s = 0; s < NSET; ++s)
    for (double** p : {&A[s], &B[s], &C[s]}) {
      CK(hipMalloc(p, dd * 8));
      for (auto& x : h) x = nd(rng);
      CK(hipMemcpy(*p, h.data(), dd * 8, hipMemcpyHostToDevice));
    }
  auto op = [&](int s) {
    vbk::GemmOp g{};
    g.M = g.N = g.K = D;
    g.A = A[s]; g.lda = D; g.B = B[s]; g.ldb = D; g.C = C[s]; g.ldc = D;
    g.alpha = 1.0;
    g.sym = sym;
    return g;
  };
  for (int r = 0; r < 60; ++r) CK(vbk::gemm(op(r % NSET), 0));
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> ts(1024 * 16);
  CK(hipMemcpyFromSymbol(ts.data(), HIP_SYMBOL(vbk::gemm_detail::g_gemm_ts), ts.size() * 8));
  const int nb = sym ? 136 : 256;
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < nb; ++b) { t0 = std::min(t0, ts[b * 16]); t1 = std::max(t1, ts[b * 16 + 15]); }
  printf("blocks %d  span (first entry -> last end) %.2f us\n", nb, (t1 - t0) * 0.01);
  // per phase: mean over blocks of (phase - entry), and of entry - t0
  double ent = 0, ph[16] = {0};
  for (int b = 0; b < nb; ++b) {
    ent += (ts[b * 16] - t0) * 0.01;
    for (int k = 1; k < 16; ++k) ph[k] += ((double)ts[b * 16 + k] - (double)ts[b * 16]) * 0.01;
  }
  printf("entry after first block: mean %.2f us\n", ent / nb);
  const char* nm[16] = {"entry", "skip done", "loop start", "k0", "k1", "k2", "k3", "k4", "k5", "k6", "k7",
                        "k-part reduced", "tile stored", "partials done", "loop end", "epilogue end"};
  const int order[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 14, 11, 12, 13, 15};
  for (int k : order) printf("  %-14s %7.2f us after entry (mean over blocks)\n", nm[k], ph[k] / nb);
  return 0;
}

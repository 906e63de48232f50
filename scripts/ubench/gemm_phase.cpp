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
  // mode 1: the Newton-Schulz T product's epilogue (device alpha and shift, diag,
  // squared-residual partials)
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  double *scal, *part;
  CK(hipMalloc(&scal, 64));
  CK(hipMalloc(&part, 4 * 256 * 8));
  {
    const double hs[2] = {-0.9, 2.1};
    CK(hipMemcpy(scal, hs, 16, hipMemcpyHostToDevice));
  }
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
    if (mode == 1) {
      g.alpha_dev = scal;
      g.sq_shift_dev = scal + 1;
      g.diag = 3.0;
      g.sq_part = part;
    }
    return g;
  };
  for (int r = 0; r < 60; ++r) CK(vbk::gemm(op(r % NSET), 0));
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> ts(1024 * 24);
  CK(hipMemcpyFromSymbol(ts.data(), HIP_SYMBOL(vbk::gemm_detail::g_gemm_ts), ts.size() * 8));
  const int nb = sym ? 136 : 256;
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < nb; ++b) { t0 = std::min(t0, ts[b * 24]); t1 = std::max(t1, ts[b * 24 + 15]); }
  printf("blocks %d  span (first entry -> last end) %.2f us\n", nb, (t1 - t0) * 0.01);
  // per phase: mean over blocks of (phase - entry), and of entry - t0
  double ent = 0, ph[24] = {0};
  for (int b = 0; b < nb; ++b) {
    ent += (ts[b * 24] - t0) * 0.01;
    for (int k = 1; k < 24; ++k) ph[k] += ((double)ts[b * 24 + k] - (double)ts[b * 24]) * 0.01;
  }
  printf("entry after first block: mean %.2f us\n", ent / nb);
  const char* nm[20] = {"entry", "skip done", "loop start", "k0", "k1", "k2", "k3", "k4", "k5", "k6", "k7",
                        "k-part reduced", "tile stored", "partials done", "loop end", "epilogue end",
                        "acc summed", "epi operands", "store pass 2 start", "store pass 2 end"};
  const int order[19] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 14, 16, 11, 17, 12, 13, 15, 18, 19};
  for (int k : order) printf("  %-14s %7.2f us after entry (mean over blocks)\n", nm[k], ph[k] / nb);
  return 0;
}

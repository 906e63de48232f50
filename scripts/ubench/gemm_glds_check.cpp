// A/B of the fp64 GEMM main loops (vb_gemm.hpp): register-staged vs LDS-DMA
// (global_load_lds).  Both must give BITWISE-identical C (same k order); then
// the mean time per launch over cold operand sets (8 sets cycled, > one XCD's
// L2) for the shapes of the full-rank step.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_glds_check.cpp -o gemm_glds_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../viabel_amd/csrc/vb_gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Shape { const char* name; int M, N, K; bool ta, tb; int group; };

int main() {
  const int NSET = 8, reps = 300;
  const size_t cap = (size_t)512 * 512;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  std::vector<double> h(cap);
  double *A[NSET], *B[NSET], *C[NSET], *C2[NSET];
  for (int s = 0; s < NSET; ++s) {
    for (double** p : {&A[s], &B[s], &C[s], &C2[s]}) {
      CK(hipMalloc(p, cap * 8));
      for (auto& x : h) x = nd(rng);
      CK(hipMemcpy(*p, h.data(), cap * 8, hipMemcpyHostToDevice));
    }
  }
  const Shape shapes[] = {{"NN 512^3", 512, 512, 512, false, false, 1},
                          {"NT 512^3", 512, 512, 512, false, true, 1},
                          {"TN 512^3", 512, 512, 512, true, false, 1},
                          {"NN 512^3 x2 grouped", 512, 512, 512, false, false, 2},
                          {"NN 128x512x512", 128, 512, 512, false, false, 1},
                          {"NN 512x512x128", 512, 512, 128, false, false, 1}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad = 0;
  for (const Shape& sh : shapes) {
    auto op = [&](int s, double* out) {
      vbk::GemmOp g{};
      g.ta = sh.ta; g.tb = sh.tb; g.M = sh.M; g.N = sh.N; g.K = sh.K;
      g.A = A[s]; g.lda = sh.ta ? sh.M : sh.K;
      g.B = B[s]; g.ldb = sh.tb ? sh.K : sh.N;
      g.C = out; g.ldc = sh.N; g.alpha = 1.0;
      return g;
    };
    auto launch = [&](int s, double* const* out) {
      vbk::GemmOp g2[2] = {op(s % NSET, out[s % NSET]), op((s + 3) % NSET, out[(s + 3) % NSET])};
      return vbk::gemm_group(g2, sh.group, 0);
    };
    // bitwise check: old loop -> C, LDS-DMA loop -> C2
    vbk::gemm_glds_enable = false;
    CK(launch(0, C));
    vbk::gemm_glds_enable = true;
    CK(launch(0, C2));
    CK(hipDeviceSynchronize());
    std::vector<double> c1((size_t)sh.M * sh.N), c2(c1.size());
    CK(hipMemcpy(c1.data(), C[0], c1.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c2.data(), C2[0], c2.size() * 8, hipMemcpyDeviceToHost));
    const bool same = memcmp(c1.data(), c2.data(), c1.size() * 8) == 0;
    bad += !same;
    float ms[2];
    for (int mode = 0; mode < 2; ++mode) {
      vbk::gemm_glds_enable = mode == 1;
      for (int r = 0; r < 40; ++r) CK(launch(r, mode ? C2 : C));
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) CK(launch(r, mode ? C2 : C));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms[mode], e0, e1));
    }
    printf("%-22s bitwise %s   regstage %7.2f us   glds %7.2f us   (%.2fx)\n", sh.name,
           same ? "SAME" : "DIFF", ms[0] * 1e3 / reps, ms[1] * 1e3 / reps, ms[0] / ms[1]);
  }
  printf("gs=%d %s\n", vbk::gemm_detail::GS, bad ? "MISMATCH" : "all bitwise identical");
  return bad ? 2 : 0;
}

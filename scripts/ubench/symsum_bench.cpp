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

// XCD-grouped block order (D = 512): block b runs on XCD b % 8 (round-robin
// dispatch); tab[b] is the geo() unit it computes, so that each XCD's 32 units
// form one band block (a, b) of the 4 x 4 grid of 128-row bands (a < b), or two
// diagonal band blocks: its operand lines shrink from all of A and X to ~1-3 MB.
template <int KT>
__global__ __launch_bounds__(vbk::symsum::NTH) void symsum_remap_kernel(const double* A, const double* X,
                                                                     int D, double alpha, double* C,
                                                                     const int* tab) {
  using namespace vbk::symsum;
  extern __shared__ double lds[];
  const Geo g = geo(tab[blockIdx.x], D / 32);
  product<KT>(A, X, D, g, lds);
  const double* vt = lds + RED;
  const int t = threadIdx.x;
  for (int e = t; e < (g.diag ? 1024 : 512); e += NTH) {
    const int r = e >> 5, c = e & 31;
    C[(long long)(g.r0 + r) * D + g.c0 + c] = alpha * vt[r * VS + c];
  }
  if (!g.diag) {
    const int c = t >> 4, r = t & 15;
    C[(long long)(g.c0 + c) * D + g.r0 + r] = alpha * vt[r * VS + c];
  }
}

static std::vector<int> xcd_table(int nt) {
  // host copy of geo(): unit -> (r0, c0)
  const int no = nt * (nt - 1) / 2, nb = nt * nt, band = nt / 4;
  std::vector<std::vector<int>> grp(8);
  for (int b = 0; b < nb; ++b) {
    int bi, bj;
    if (b < 2 * no) {
      int t = b >> 1, i = 0;
      while (t >= nt - 1 - i) { t -= nt - 1 - i; ++i; }
      bi = i; bj = i + 1 + t;
    } else {
      bi = bj = b - 2 * no;
    }
    const int ra = bi / band, cb = bj / band;
    int gi;
    if (ra == cb) gi = (ra == 0 || ra == 3) ? 6 : 7;
    else {   // (0,1) (0,2) (0,3) (1,2) (1,3) (2,3) -> 0..5
      static const int id[4][4] = {{-1, 0, 1, 2}, {-1, -1, 3, 4}, {-1, -1, -1, 5}, {-1, -1, -1, -1}};
      gi = id[ra][cb];
    }
    grp[gi].push_back(b);
  }
  std::vector<int> tab(nb);
  for (int x = 0; x < 8; ++x) {
    if ((int)grp[x].size() != nb / 8) { printf("group %d has %zu units\n", x, grp[x].size()); exit(1); }
    for (int q = 0; q < nb / 8; ++q) tab[8 * q + x] = grp[x][q];
  }
  return tab;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int D = argc > 1 ? atoi(argv[1]) : 512;
  const int NSET = argc > 3 ? atoi(argv[3]) : 8, reps = 200;
  if (NSET < 1 || NSET > 8) { printf("nset in [1, 8]\n"); return 1; }
  const size_t dd = (size_t)D * D;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::vector<double> h(dd);
  double *A[8], *X[8], *C[8];
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
  int* dtab = nullptr;
  if (D == 512) {
    const std::vector<int> tab = xcd_table(D / 32);
    CK(hipMalloc(&dtab, tab.size() * sizeof(int)));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(symsum_remap_kernel<128>, dim3(256), dim3(vbk::symsum::NTH),
                       vbk::symsum::Cfg<128>::LDS_BYTES, 0, A[0], X[0], D, 1.0, C[0], (const int*)dtab);
    CK(hipDeviceSynchronize());
    std::vector<double> c1(dd), a1(dd), x1(dd);
    CK(hipMemcpy(c1.data(), C[0], dd * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(a1.data(), A[0], dd * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(x1.data(), X[0], dd * 8, hipMemcpyDeviceToHost));
    double e1 = 0.0;
    for (int i = 0; i < D; i += 7)
      for (int j = 0; j < D; ++j) {
        double r = 0.0;
        for (int k = 0; k < D; ++k) r += a1[(size_t)i * D + k] * x1[(size_t)k * D + j] + x1[(size_t)i * D + k] * a1[(size_t)k * D + j];
        e1 = fmax(e1, fabs(r - c1[(size_t)i * D + j]) / (1.0 + fabs(r)));
      }
    printf("xcd-grouped order: max rel err %.3e (every 7th row)\n", e1);
  }
  for (int mode = 0; mode < 3; ++mode) {
    if (mode == 2 && !dtab) break;
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
        } else if (mode == 1) {
          CK(vbk::symsum::plain(A[s], X[s], D, 1.0, C[s], 0, kt));
        } else {
          hipLaunchKernelGGL(symsum_remap_kernel<128>, dim3(256), dim3(vbk::symsum::NTH),
                             vbk::symsum::Cfg<128>::LDS_BYTES, 0, A[s], X[s], D, 1.0, C[s],
                             (const int*)dtab);
        }
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      static const char* nm[3] = {"plain gemm A X", "symsum A X + X A", "symsum, xcd-grouped order"};
      if (pass) printf("%s (nset %d): %.2f us per launch\n", nm[mode], NSET, 1e3 * ms / reps);
    }
  }
  return 0;
}

// Time rocSOLVER symmetric eigensolvers at n = 512 (fp64) on one MI355X:
// dsyevd and dsyevj on a random SPD matrix, and dsyevj on a nearly diagonal
// matrix (the warm-start case: A = V^T Sigma V with the previous step's V).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

static double now_ms(hipEvent_t a, hipEvent_t b) { float ms; hipEventElapsedTime(&ms, a, b); return ms; }

int main() {
  const int n = 512;
  std::vector<double> h(n * n), g(n * n);
  srand(3);
  for (auto& v : g) v = (rand() / (double)RAND_MAX - 0.5);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int k = 0; k < n; ++k) s += g[i * n + k] * g[j * n + k];
      h[i * n + j] = s / n + (i == j ? 1.0 : 0.0);
    }
  std::vector<double> nd(n * n, 0.0);
  for (int i = 0; i < n; ++i) {
    nd[i * n + i] = 1.0 + i * 0.01;
    for (int j = 0; j < n; ++j) if (i != j) nd[i * n + j] = 1e-4 * (g[i * n + j] + g[j * n + i]);
  }
  rocblas_handle hd; rocblas_create_handle(&hd);
  double *dA, *dW, *dE, *dres; rocblas_int *dinfo, *dsw;
  (void)hipMalloc(&dA, sizeof(double) * n * n); (void)hipMalloc(&dW, sizeof(double) * n);
  (void)hipMalloc(&dE, sizeof(double) * n); (void)hipMalloc(&dres, sizeof(double));
  (void)hipMalloc(&dinfo, sizeof(int)); (void)hipMalloc(&dsw, sizeof(int));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int t = 0; t < 3; ++t) {
    for (int rep = 0; rep < 3; ++rep) {
      const std::vector<double>& src = (t == 2) ? nd : h;
      (void)hipMemcpy(dA, src.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      if (t == 0)
        rocsolver_dsyevd(hd, rocblas_evect_original, rocblas_fill_lower, n, dA, n, dW, dE, dinfo);
      else
        rocsolver_dsyevj(hd, rocblas_esort_none, rocblas_evect_original, rocblas_fill_lower, n, dA, n,
                         1e-14, dres, 100, dsw, dW, dinfo);
      hipEventRecord(e1); hipEventSynchronize(e1);
      int sw = 0, info = 0; (void)hipMemcpy(&sw, dsw, 4, hipMemcpyDeviceToHost); (void)hipMemcpy(&info, dinfo, 4, hipMemcpyDeviceToHost);
      if (rep == 2) printf("%s: %.3f ms (info %d, sweeps %d)\n",
                           t == 0 ? "dsyevd random SPD" : t == 1 ? "dsyevj random SPD" : "dsyevj near-diagonal",
                           now_ms(e0, e1), info, t ? sw : -1);
    }
  }
  return 0;
}

// vb_rhat.hip — convergence diagnostics over optimisation histories
// (viabel/functions.py:8-77): split-chain R-hat over batches of iteration
// segments, and stochastic iterate averaging (cumulative means).
#include "vb_device.hpp"
#include "vb_internal.hpp"

namespace vbk {
using namespace vbd;

namespace {

// One thread per (job, parameter).  compute_R_hat on chains[:, s:s+len, :]:
// the segment is split into halves (psi = 2 nc half-chains of h = len/2 draws),
// two-pass means / variances as numpy does, then
//   B = h sum_j (mean_j - mean)^2 / (2nc - 1),  W = mean_j s_j^2 + 1e-8,
//   var_hat = (h - 1) / h + B / (h W),  R-hat = sqrt(var_hat).
__global__ __launch_bounds__(256) void rhat_kernel(const double* chains, long long nc, long long n,
                                                   long long P, const long long* start,
                                                   const long long* len, double* var_out,
                                                   double* rhat_out) {
  const long long job = blockIdx.y;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const long long s0 = start[job], h = len[job] / 2;
  const long long nc2 = 2 * nc;
  double sum_means = 0.0, sum_var = 0.0;
  long long n_var = 0;
  // pass 1: grand mean of the half-chain means
  for (long long j = 0; j < nc2; ++j) {
    const double* x = chains + ((j >> 1) * n + s0 + (j & 1) * h) * P + p;
    double m = 0.0;
    for (long long t = 0; t < h; ++t) m += x[t * P];
    sum_means += m / (double)h;
  }
  const double grand = sum_means / (double)nc2;
  double B = 0.0;
  for (long long j = 0; j < nc2; ++j) {
    const double* x = chains + ((j >> 1) * n + s0 + (j & 1) * h) * P + p;
    double m = 0.0;
    for (long long t = 0; t < h; ++t) m += x[t * P];
    m /= (double)h;
    double ss = 0.0;
    for (long long t = 0; t < h; ++t) {
      const double d = x[t * P] - m;
      ss += d * d;
    }
    const double sj = ss / (double)(h - 1);
    if (!isnan(sj)) {  // np.nanmean over the half-chain variances
      sum_var += sj;
      ++n_var;
    }
    B += (m - grand) * (m - grand);
  }
  B = (double)h * B / (double)(nc2 - 1);
  const double W = sum_var / (double)n_var + 1e-8;
  const double vh = (double)(h - 1) / (double)h + B / ((double)h * W);
  if (var_out) var_out[job * P + p] = vh;
  rhat_out[job * P + p] = sqrt(vh);
}

// out[t][c] = mean of x[start..start+t][c]  (np.cumsum order, then / (t + 1))
__global__ __launch_bounds__(256) void iterate_average_kernel(const double* x, long long n,
                                                              long long ld, long long cols,
                                                              long long start, double* out) {
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  double acc = 0.0;
  for (long long t = start; t < n; ++t) {
    acc += x[t * ld + c];
    out[(t - start) * cols + c] = acc / (double)(t - start + 1);
  }
}

}  // namespace

hipError_t launch_rhat(const double* chains, long long nc, long long n, long long P,
                       long long n_jobs, const long long* start, const long long* len,
                       double* var_out, double* rhat_out, hipStream_t s) {
  if (n_jobs <= 0 || P <= 0) return hipSuccess;
  hipLaunchKernelGGL(rhat_kernel, dim3((unsigned)((P + 255) / 256), (unsigned)n_jobs), dim3(256), 0,
                     s, chains, nc, n, P, start, len, var_out, rhat_out);
  return hipGetLastError();
}

hipError_t launch_iterate_average(const double* x, long long n, long long ld, long long cols,
                                  long long start, double* out, hipStream_t s) {
  if (cols <= 0 || n <= start) return hipSuccess;
  hipLaunchKernelGGL(iterate_average_kernel, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, s,
                     x, n, ld, cols, start, out);
  return hipGetLastError();
}

}  // namespace vbk

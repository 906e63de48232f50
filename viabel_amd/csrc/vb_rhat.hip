// vb_rhat.hip — convergence diagnostics over optimisation histories
// (viabel/functions.py:8-77): split-chain R-hat over batches of iteration
// segments, and stochastic iterate averaging (cumulative means).
#include "vb_device.hpp"
#include "vb_internal.hpp"

namespace vbk {
using namespace vbd;

namespace {

// compute_R_hat on chains[:, s:s+len, :] (functions.py:8-31) in two stages, so
// that chains held by different ranks combine to the same bits as one process:
//   rhat_stats_kernel    one thread per (job, half-chain j, parameter): the
//                        half-chain mean m_j = (sum of its h = len/2 draws) / h and
//                        the centred sum of squares ss_j = sum (x - m_j)^2 (numpy's
//                        two-pass np.mean / squared deviations);
//   rhat_combine_kernel  one thread per (job, parameter), half-chains in order:
//                        grand = sum_j m_j / (2 nc), s_j^2 = ss_j / (h - 1),
//                        B = h sum_j (m_j - grand)^2 / (2 nc - 1),
//                        W = nanmean_j s_j^2 + 1e-8,
//                        var_hat = (h - 1) / h + B / (h W), R-hat = sqrt(var_hat).
// Half-chain j of chain c is j = 2c + h (np.reshape of [nc][2h][P] into
// [2nc][h][P]); stats are [job][2 nc][P].
__global__ __launch_bounds__(256) void rhat_stats_kernel(const double* chains, long long n,
                                                         long long P, const long long* start,
                                                         const long long* len, double* mean_out,
                                                         double* ss_out) {
  const long long job = blockIdx.y, j = blockIdx.z, nc2 = gridDim.z;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const long long h = len[job] / 2;
  const double* x = chains + ((j >> 1) * n + start[job] + (j & 1) * h) * P + p;
  double m = 0.0;
  for (long long t = 0; t < h; ++t) m += x[t * P];
  m /= (double)h;
  double ss = 0.0;
  for (long long t = 0; t < h; ++t) {
    const double d = x[t * P] - m;
    ss += d * d;
  }
  const long long o = (job * nc2 + j) * P + p;
  mean_out[o] = m;
  ss_out[o] = ss;
}

__global__ __launch_bounds__(256) void rhat_combine_kernel(const double* mean, const double* ss,
                                                           long long nc2, long long P,
                                                           const long long* len, double* var_out,
                                                           double* rhat_out) {
  const long long job = blockIdx.y;
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const long long h = len[job] / 2;
  const double* mj = mean + job * nc2 * P + p;
  const double* sj = ss + job * nc2 * P + p;
  double sum_means = 0.0;
  for (long long j = 0; j < nc2; ++j) sum_means += mj[j * P];
  const double grand = sum_means / (double)nc2;
  double B = 0.0, sum_var = 0.0;
  long long n_var = 0;
  for (long long j = 0; j < nc2; ++j) {
    const double m = mj[j * P];
    const double v = sj[j * P] / (double)(h - 1);
    if (!isnan(v)) {  // np.nanmean over the half-chain variances
      sum_var += v;
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

hipError_t launch_rhat_stats(const double* chains, long long nc, long long n, long long P,
                             long long n_jobs, const long long* start, const long long* len,
                             double* mean_out, double* ss_out, hipStream_t s) {
  if (n_jobs <= 0 || P <= 0 || nc <= 0) return hipSuccess;
  hipLaunchKernelGGL(rhat_stats_kernel,
                     dim3((unsigned)((P + 255) / 256), (unsigned)n_jobs, (unsigned)(2 * nc)),
                     dim3(256), 0, s, chains, n, P, start, len, mean_out, ss_out);
  return hipGetLastError();
}

hipError_t launch_rhat_combine(const double* mean, const double* ss, long long nc2, long long P,
                               long long n_jobs, const long long* len, double* var_out,
                               double* rhat_out, hipStream_t s) {
  if (n_jobs <= 0 || P <= 0) return hipSuccess;
  hipLaunchKernelGGL(rhat_combine_kernel, dim3((unsigned)((P + 255) / 256), (unsigned)n_jobs),
                     dim3(256), 0, s, mean, ss, nc2, P, len, var_out, rhat_out);
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

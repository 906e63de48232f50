// vb_bounds.hip — importance-weight reductions behind viabel.bounds.
//
//   divergence_bound         viabel/bounds.py:142-180
//   mean_and_check_mc_error  viabel/bounds.py:183-192   (mean, std/sqrt(n))
//   wasserstein moments      viabel/bounds.py:127-135   (centred 2p-th moments)
//   np.cov(samples.T)        viabel/bounds.py:55-56
//
// Every reduction is a fixed-order two-level tree (per-block partials, then one
// block combines them in block order), so results are bitwise reproducible
// run to run.  Passes follow numpy's two-pass definitions (np.std centres on
// the mean first) rather than one-pass power sums, which cancel badly.
#include <algorithm>
#include <cstdlib>

#include "vb_device.hpp"
#include "vb_internal.hpp"

using namespace vbd;

namespace vbk {

namespace {

constexpr int kRedBlocks = 1024;
// divergence scratch per log-weight row: partials [4 kRedBlocks] (two-pass form;
// the three-pass form uses 2 per block), sc [4], m2 [2] (+ pad)
constexpr long long kDivStride = 4 * kRedBlocks + 8;

__device__ __forceinline__ double block_sum1(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ double block_max1(double v, double* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double r = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return r;
}

__global__ void set_scalar_kernel(double* p, double v) { *p = v; }

// VIABEL_AMD_DIV_TWO_PASS=0: the three-pass divergence statistics (numpy's two-pass
// definitions) at every size instead of the two-pass Welford / Chan form from
// kDivTwoPassMinN log weights on (A/B and parity switch; the two agree to rounding)
constexpr long long kDivTwoPassMinN = 1LL << 16;
bool div_two_pass_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_DIV_TWO_PASS");
    return !(e && e[0] == '0');
  }();
  return on;
}

int red_grid(long long n) {
  long long g = (n + 2047) / 2048;
  if (g < 1) g = 1;
  if (g > kRedBlocks) g = kRedBlocks;
  return (int)g;
}

// pass 1: per-block max and sum of lw
__global__ __launch_bounds__(256) void lw_max_sum_kernel(const double* lw, long long n,
                                                         double* part, long long ld) {
  __shared__ double red[4];
  lw += (long long)blockIdx.y * ld;
  part += (long long)blockIdx.y * kDivStride;
  double m = -INFINITY, s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const double v = lw[i];
    m = fmax(m, v);
    s += v;
  }
  m = block_max1(m, red);
  s = block_sum1(s, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = m;
    part[2 * blockIdx.x + 1] = s;
  }
}

// combine pass-1 partials: sc[0] = max, sc[1] = mean
__global__ __launch_bounds__(256) void lw_max_sum_final(const double* part, int nb, long long n,
                                                        double* sc) {
  __shared__ double red[4];
  part += (long long)blockIdx.y * kDivStride;
  sc += (long long)blockIdx.y * kDivStride;
  double m = -INFINITY, s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) {
    m = fmax(m, part[2 * b]);
    s += part[2 * b + 1];
  }
  m = block_max1(m, red);
  s = block_sum1(s, red);
  if (threadIdx.x == 0) {
    sc[0] = m;
    sc[1] = s / (double)n;
  }
}

// pass 2: sum of r = exp(lw - max)^alpha and of (lw - mean)^2
__global__ __launch_bounds__(256) void lw_rescaled_kernel(const double* lw, long long n,
                                                          double alpha, const double* sc,
                                                          double* part, long long ld) {
  __shared__ double red[4];
  lw += (long long)blockIdx.y * ld;
  sc += (long long)blockIdx.y * kDivStride;
  part += (long long)blockIdx.y * kDivStride;
  const double mx = sc[0], mean = sc[1];
  double s = 0.0, q = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const double v = lw[i];
    const double e = exp(v - mx);
    s += (alpha == 2.0) ? e * e : pow(e, alpha);
    const double dv = v - mean;
    q += dv * dv;
  }
  s = block_sum1(s, red);
  q = block_sum1(q, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = q;
  }
}

__global__ __launch_bounds__(256) void sum2_final(const double* part, int nb, long long n,
                                                  double* out2) {
  __shared__ double red[4];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nb; k += 256) {
    a += part[2 * k];
    b += part[2 * k + 1];
  }
  a = block_sum1(a, red);
  b = block_sum1(b, red);
  if (threadIdx.x == 0) {
    out2[0] = a / (double)n;
    out2[1] = b / (double)n;
  }
}

// sum2_final for the divergence rows (partials and result at the row's scratch)
__global__ __launch_bounds__(256) void div_sum2_final(const double* part, int nb, long long n,
                                                      double* out2) {
  part += (long long)blockIdx.y * kDivStride;
  out2 += (long long)blockIdx.y * kDivStride;
  __shared__ double red[4];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nb; k += 256) {
    a += part[2 * k];
    b += part[2 * k + 1];
  }
  a = block_sum1(a, red);
  b = block_sum1(b, red);
  if (threadIdx.x == 0) {
    out2[0] = a / (double)n;
    out2[1] = b / (double)n;
  }
}

// pass 3: sum of (r - mean_r)^2
__global__ __launch_bounds__(256) void lw_rdev_kernel(const double* lw, long long n, double alpha,
                                                      const double* sc, const double* m2,
                                                      double* part, long long ld) {
  __shared__ double red[4];
  lw += (long long)blockIdx.y * ld;
  sc += (long long)blockIdx.y * kDivStride;
  m2 += (long long)blockIdx.y * kDivStride;
  part += (long long)blockIdx.y * kDivStride;
  const double mx = sc[0], mr = m2[0];
  double q = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const double e = exp(lw[i] - mx);
    const double r = (alpha == 2.0) ? e * e : pow(e, alpha);
    q += (r - mr) * (r - mr);
  }
  q = block_sum1(q, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = q;
    part[2 * blockIdx.x + 1] = 0.0;
  }
}

// ---- two passes over the log weights (bounds_divergence_rows, n >= 2^16) -------
// Every statistic divergence_bound needs (bounds.py:142-192) from TWO reads of lw
// instead of three: pass A the max M and Welford (count, mean, M2) of lw; pass B
// Welford of r = exp(alpha (lw - M)).  Thread states merge with Chan et al.'s
// pairwise formula (Am. Stat. 37 (1983) 242-247) in a fixed order (a shuffle-down
// tree in each wave, waves in order, blocks in order), so the results are bitwise
// reproducible; against numpy's two-pass np.mean / np.std they differ by rounding
// (as any reduction order at these sizes does).  Each thread streams kDivPer log
// weights (four loads in flight), so the merges are a small part of the pass.
struct Welf {
  double n, mean, m2;
};

__device__ __forceinline__ void welf_add(Welf& a, double v) {
  a.n += 1.0;
  double inv = __builtin_amdgcn_rcp(a.n);          // 1 / count, refined (~1 ulp)
  inv = fma(inv, fma(-a.n, inv, 1.0), inv);
  inv = fma(inv, fma(-a.n, inv, 1.0), inv);
  const double d = v - a.mean;
  a.mean = fma(d, inv, a.mean);
  a.m2 = fma(d, v - a.mean, a.m2);
}

__device__ __forceinline__ Welf welf_merge(const Welf& a, const Welf& b) {
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  Welf o;
  o.n = a.n + b.n;
  const double wb = b.n / o.n;
  const double d = b.mean - a.mean;
  o.mean = fma(d, wb, a.mean);
  o.m2 = fma(d * d, a.n * wb, a.m2 + b.m2);
  return o;
}

__device__ __forceinline__ Welf welf_shfl_down(const Welf& a, int off) {
  return Welf{__shfl_down(a.n, off, 64), __shfl_down(a.mean, off, 64), __shfl_down(a.m2, off, 64)};
}

constexpr int kDivPer = 32;   // log weights per thread per pass
int div2_grid(long long n) {
  long long g = (n + 256LL * kDivPer - 1) / (256LL * kDivPer);
  return (int)std::max(1LL, std::min<long long>(g, kRedBlocks));
}

// the block's Welford state (+ max) in a fixed order; lane 0 of wave 0 returns it
template <bool MAX>
__device__ __forceinline__ Welf welf_block(Welf a, double& m, Welf* red, double* redm) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a = welf_merge(a, welf_shfl_down(a, off));
    if (MAX) m = fmax(m, __shfl_down(m, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = a;
    if (MAX) redm[threadIdx.x >> 6] = m;
  }
  __syncthreads();
  if (MAX) m = fmax(fmax(redm[0], redm[1]), fmax(redm[2], redm[3]));
  return welf_merge(welf_merge(red[0], red[1]), welf_merge(red[2], red[3]));
}

// grid-stride loads of this thread's log weights, four in flight
template <class F>
__device__ __forceinline__ void div_stream(const double* lw, long long n, F&& f) {
  const long long st = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = lw[i + u * st];
#pragma unroll
    for (int u = 0; u < 4; ++u) f(v[u]);
  }
  for (; i < n; i += st) f(lw[i]);
}

// pass A: partials [4 b .. 4 b + 3] = (max, n, mean, M2) of lw
__global__ __launch_bounds__(256) void lw_div_a_kernel(const double* lw, long long n, double* part,
                                                       long long ld) {
  __shared__ Welf red[4];
  __shared__ double redm[4];
  lw += (long long)blockIdx.y * ld;
  part += (long long)blockIdx.y * kDivStride;
  Welf a{0.0, 0.0, 0.0};
  double m = -INFINITY;
  div_stream(lw, n, [&](double v) {
    m = fmax(m, v);
    welf_add(a, v);
  });
  const Welf b = welf_block<true>(a, m, red, redm);
  if (threadIdx.x == 0) {
    double* o = part + 4 * blockIdx.x;
    o[0] = m;
    o[1] = b.n;
    o[2] = b.mean;
    o[3] = b.m2;
  }
}

// merge pass A's block states in block order: sc[0] = max, sc[1] = mean, sc[2] = M2
__global__ __launch_bounds__(64) void div_a_final(const double* part, int nb, double* sc) {
  part += (long long)blockIdx.y * kDivStride;
  sc += (long long)blockIdx.y * kDivStride;
  Welf a{0.0, 0.0, 0.0};
  double m = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += 64) {
    const double* q = part + 4 * b;
    m = fmax(m, q[0]);
    a = welf_merge(a, Welf{q[1], q[2], q[3]});
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    a = welf_merge(a, welf_shfl_down(a, off));
    m = fmax(m, __shfl_down(m, off, 64));
  }
  if (threadIdx.x == 0) {
    sc[0] = m;
    sc[1] = a.mean;
    sc[2] = a.m2;
  }
}

// pass B: partials [3 b ..] = Welford (n, mean, M2) of r = exp(alpha (lw - max))
__global__ __launch_bounds__(256) void lw_div_b_kernel(const double* lw, long long n, double alpha,
                                                       const double* sc, double* part,
                                                       long long ld) {
  __shared__ Welf red[4];
  lw += (long long)blockIdx.y * ld;
  sc += (long long)blockIdx.y * kDivStride;
  part += (long long)blockIdx.y * kDivStride;
  const double mx = sc[0];
  Welf a{0.0, 0.0, 0.0};
  div_stream(lw, n, [&](double v) { welf_add(a, exp_fast(alpha * (v - mx))); });
  double unused = 0.0;
  const Welf b = welf_block<false>(a, unused, red, nullptr);
  if (threadIdx.x == 0) {
    double* o = part + 3 * blockIdx.x;
    o[0] = b.n;
    o[1] = b.mean;
    o[2] = b.m2;
  }
}

// merge pass B's block states; out7 as divergence_final
__global__ __launch_bounds__(64) void div_b_final(const double* part, int nb, long long n,
                                                  double alpha, int has_elbo, double elbo,
                                                  const double* sc, double* out7) {
  part += (long long)blockIdx.y * kDivStride;
  sc += (long long)blockIdx.y * kDivStride;
  out7 += (long long)blockIdx.y * 7;
  Welf a{0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nb; b += 64) {
    const double* q = part + 3 * b;
    a = welf_merge(a, Welf{q[0], q[1], q[2]});
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) a = welf_merge(a, welf_shfl_down(a, off));
  if (threadIdx.x == 0) {
    const double sq = sqrt((double)n);
    const double mean_r = a.mean;
    const double se_r = sqrt(a.m2 / (double)n) / sq;
    const double cubo = log(mean_r) / alpha + sc[0];
    const double mean_lw = sc[1];
    const double se_lw = has_elbo ? NAN : sqrt(sc[2] / (double)n) / sq;
    const double lnb = has_elbo ? elbo : mean_lw;
    out7[0] = alpha / (alpha - 1.0) * (cubo - lnb);
    out7[1] = lnb;
    out7[2] = mean_r;
    out7[3] = se_r;
    out7[4] = mean_lw;
    out7[5] = se_lw;
    out7[6] = sc[0];
  }
}

// out7: d_alpha, elbo, mean_r, se_r, mean_lw, se_lw, log max
__global__ void divergence_final(const double* part, int nb, long long n, double alpha,
                                 int has_elbo, double elbo, const double* sc, const double* m2,
                                 double* out7) {
  __shared__ double red[4];
  part += (long long)blockIdx.y * kDivStride;
  sc += (long long)blockIdx.y * kDivStride;
  m2 += (long long)blockIdx.y * kDivStride;
  out7 += (long long)blockIdx.y * 7;
  double q = 0.0;
  for (int k = threadIdx.x; k < nb; k += 256) q += part[2 * k];
  q = block_sum1(q, red);
  if (threadIdx.x == 0) {
    const double sq = sqrt((double)n);
    const double mean_r = m2[0];
    const double se_r = sqrt(q / (double)n) / sq;
    const double cubo = log(mean_r) / alpha + sc[0];
    const double mean_lw = sc[1];
    const double se_lw = has_elbo ? NAN : sqrt(m2[1]) / sq;
    const double lnb = has_elbo ? elbo : mean_lw;
    out7[0] = alpha / (alpha - 1.0) * (cubo - lnb);
    out7[1] = lnb;
    out7[2] = mean_r;
    out7[3] = se_r;
    out7[4] = mean_lw;
    out7[5] = se_lw;
    out7[6] = sc[0];
  }
}

// ---- column means of x [n][d] ---------------------------------------------
// grid (row chunks, column tiles of 64); block = 64 columns x 4 row lanes
__global__ __launch_bounds__(256) void col_sum_kernel(const double* x, long long n, long long d,
                                                      long long rows_per_chunk, double* part,
                                                      const double* w = nullptr) {
  __shared__ double red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const long long col = (long long)blockIdx.y * 64 + cl;
  const long long r0 = (long long)blockIdx.x * rows_per_chunk;
  const long long r1 = min(n, r0 + rows_per_chunk);
  double s = 0.0;
  if (col < d)
    for (long long r = r0 + rl; r < r1; r += 4) s += w ? w[r] * x[r * d + col] : x[r * d + col];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && col < d)
    part[(long long)blockIdx.x * d + col] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// mean = column sums / n, or / *sw (the weight sum on the device)
__global__ __launch_bounds__(256) void col_final_kernel(const double* part, int nchunk,
                                                        long long n, long long d, double* mean,
                                                        const double* sw = nullptr) {
  const long long col = (long long)blockIdx.x * 256 + threadIdx.x;
  if (col >= d) return;
  double s = 0.0;
  for (int k = 0; k < nchunk; ++k) s += part[(long long)k * d + col];
  mean[col] = s / (sw ? *sw : (double)n);
}

// 1-D fast path: mean of x[n]
__global__ __launch_bounds__(256) void flat_sum_kernel(const double* x, long long n,
                                                       double* part) {
  __shared__ double red[4];
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    s += x[i];
  s = block_sum1(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void flat_final_kernel(const double* part, int nb, long long n,
                                                         double* mean) {
  __shared__ double red[4];
  double s = 0.0;
  for (int k = threadIdx.x; k < nb; k += 256) s += part[k];
  s = block_sum1(s, red);
  if (threadIdx.x == 0) mean[0] = s / (double)n;
}

// ---- centred power sums over all elements ---------------------------------
__global__ __launch_bounds__(256) void cpow_kernel(const double* x, long long n, long long d,
                                                   const double* mean, double* part) {
  __shared__ double red[4];
  const long long tot = n * d;
  double s2 = 0.0, s4 = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot;
       i += (long long)gridDim.x * 256) {
    const double v = x[i] - mean[d == 1 ? 0 : i % d];
    const double v2 = v * v;
    s2 += v2;
    s4 += v2 * v2;
  }
  s2 = block_sum1(s2, red);
  s4 = block_sum1(s4, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s2;
    part[2 * blockIdx.x + 1] = s4;
  }
}

// ---- covariance: one block row per (chunk, pair) ----------------------------
__global__ __launch_bounds__(256) void cov_kernel(const double* x, long long n, long long d,
                                                  const double* mean, long long rows_per_chunk,
                                                  double* part, const double* w = nullptr) {
  __shared__ double red[4];
  const int pair = blockIdx.y;
  // pair -> (i, j), i <= j, row-major upper triangle
  int i = 0, rem = pair;
  while (rem >= d - i) {
    rem -= (int)(d - i);
    ++i;
  }
  const int j = i + rem;
  const long long r0 = (long long)blockIdx.x * rows_per_chunk;
  const long long r1 = min(n, r0 + rows_per_chunk);
  const double mi = mean[i], mj = mean[j];
  double s = 0.0;
  for (long long r = r0 + threadIdx.x; r < r1; r += 256) {
    const double c = (x[r * d + i] - mi) * (x[r * d + j] - mj);
    s += w ? w[r] * c : c;
  }
  s = block_sum1(s, red);
  if (threadIdx.x == 0) part[(long long)blockIdx.x * gridDim.y + pair] = s;
}

// cov = pair sums / (n - 1), or / *fact (np.cov's aweights normaliser, device)
__global__ __launch_bounds__(256) void cov_final_kernel(const double* part, int nchunk, int npairs,
                                                        long long n, long long d, double* cov,
                                                        const double* fact = nullptr) {
  const int pair = blockIdx.x * 256 + threadIdx.x;
  if (pair >= npairs) return;
  int i = 0, rem = pair;
  while (rem >= d - i) {
    rem -= (int)(d - i);
    ++i;
  }
  const int j = i + rem;
  double s = 0.0;
  for (int k = 0; k < nchunk; ++k) s += part[(long long)k * npairs + pair];
  const double c = s / (fact ? *fact : (double)(n - 1));
  cov[(long long)i * d + j] = c;
  cov[(long long)j * d + i] = c;
}

int col_chunks(long long n, long long* rows_per_chunk) {
  long long nc = (n + 4095) / 4096;
  if (nc < 1) nc = 1;
  if (nc > 512) nc = 512;
  *rows_per_chunk = (n + nc - 1) / nc;
  return (int)nc;
}

hipError_t means(const double* x, long long n, long long d, double* scratch, double* mean,
                 hipStream_t s) {
  if (d == 1) {
    const int g = red_grid(n);
    hipLaunchKernelGGL(flat_sum_kernel, dim3(g), dim3(256), 0, s, x, n, scratch);
    hipLaunchKernelGGL(flat_final_kernel, dim3(1), dim3(256), 0, s, scratch, g, n, mean);
  } else {
    long long rpc;
    const int nc = col_chunks(n, &rpc);
    hipLaunchKernelGGL(col_sum_kernel, dim3(nc, (unsigned)((d + 63) / 64)), dim3(256), 0, s, x, n,
                       d, rpc, scratch);
    hipLaunchKernelGGL(col_final_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s,
                       scratch, nc, n, d, mean);
  }
  return hipGetLastError();
}

}  // namespace

size_t bounds_scratch_doubles(long long n, long long d) {
  long long rpc;
  const int nc = col_chunks(n, &rpc);
  const long long npairs = d * (d + 1) / 2;
  long long need = 4LL * kRedBlocks + 16;
  need = need > nc * d + 16 ? need : nc * d + 16;
  if (d <= kCovDMax && need < nc * npairs + 16) need = nc * npairs + 16;
  return (size_t)need + 2 * (size_t)d + 16;
}

hipError_t bounds_divergence(const double* lw, long long n, double alpha, int has_elbo,
                             double elbo, double* scratch, double* out7, hipStream_t s) {
  return bounds_divergence_rows(lw, 1, n, n, alpha, has_elbo, elbo, scratch, out7, s);
}

// rows independent log-weight vectors (row r at lw + r ld) in one launch chain:
// every kernel takes its row from blockIdx.y, scratch kDivStride doubles per row
hipError_t bounds_divergence_rows(const double* lw, long long rows, long long n, long long ld,
                                  double alpha, int has_elbo, double elbo, double* scratch,
                                  double* out7, hipStream_t s) {
  if (rows < 1 || rows > 65535) return hipErrorInvalidValue;
  const int g = red_grid(n);
  const unsigned R = (unsigned)rows;
  double* part = scratch;
  double* sc = scratch + 4 * kRedBlocks;   // after the largest (two-pass) partials
  double* m2 = sc + 4;
  // below 2^16 log weights the exact three-pass form (numpy's definitions, whose
  // bits it reproduces on small inputs -- the Monte Carlo warning texts print them);
  // above, no reduction order reproduces numpy's pairwise sums bit for bit anyway,
  // and the two-pass Welford form reads the 8 B per log weight twice, not three times
  if (div_two_pass_enabled() && n >= kDivTwoPassMinN) {
    const int g2 = div2_grid(n);
    hipLaunchKernelGGL(lw_div_a_kernel, dim3(g2, R), dim3(256), 0, s, lw, n, part, ld);
    hipLaunchKernelGGL(div_a_final, dim3(1, R), dim3(64), 0, s, part, g2, sc);
    hipLaunchKernelGGL(lw_div_b_kernel, dim3(g2, R), dim3(256), 0, s, lw, n, alpha, sc, part, ld);
    hipLaunchKernelGGL(div_b_final, dim3(1, R), dim3(64), 0, s, part, g2, n, alpha, has_elbo, elbo,
                       sc, out7);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(lw_max_sum_kernel, dim3(g, R), dim3(256), 0, s, lw, n, part, ld);
  hipLaunchKernelGGL(lw_max_sum_final, dim3(1, R), dim3(256), 0, s, part, g, n, sc);
  hipLaunchKernelGGL(lw_rescaled_kernel, dim3(g, R), dim3(256), 0, s, lw, n, alpha, sc, part, ld);
  hipLaunchKernelGGL(div_sum2_final, dim3(1, R), dim3(256), 0, s, part, g, n, m2);
  hipLaunchKernelGGL(lw_rdev_kernel, dim3(g, R), dim3(256), 0, s, lw, n, alpha, sc, m2, part, ld);
  hipLaunchKernelGGL(divergence_final, dim3(1, R), dim3(256), 0, s, part, g, n, alpha, has_elbo,
                     elbo, sc, m2, out7);
  return hipGetLastError();
}

size_t bounds_divergence_scratch_doubles(long long rows) { return (size_t)(rows * kDivStride); }

hipError_t bounds_centered_moments(const double* x, long long n, long long d, double* scratch,
                                   double* out2, hipStream_t s) {
  // scratch layout: [mean (d)] [partials]
  double* mean = scratch;
  double* part = scratch + d + 8;
  hipError_t e = means(x, n, d, part, mean, s);
  if (e != hipSuccess) return e;
  const int g = red_grid(n * d);
  hipLaunchKernelGGL(cpow_kernel, dim3(g), dim3(256), 0, s, x, n, d, mean, part);
  hipLaunchKernelGGL(sum2_final, dim3(1), dim3(256), 0, s, part, g, n, out2);
  return hipGetLastError();
}

namespace {
__global__ __launch_bounds__(256) void center_kernel(const double* x, long long n, long long d,
                                                     const double* mean, double* xc) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx < n * d) xc[idx] = x[idx] - mean[idx % d];
}

// weights for np.cov(aweights) / np.average: with LOGW, w_i = exp(lw_i - max lw)
// (improve_with_psis, notebooks/experiments.py:80-82) written to wout after a
// max pass; partial sums of w and w^2 per block
template <bool LOGW>
__global__ __launch_bounds__(256) void wsum_kernel(const double* w, long long n, const double* mx,
                                                   double* wout, double* part) {
  __shared__ double red[4];
  const double m = LOGW ? *mx : 0.0;
  double a = 0.0, b = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    double v = w[i];
    if (LOGW) {
      v = exp(v - m);
      wout[i] = v;
    }
    a += v;
    b += v * v;
  }
  a = block_sum1(a, red);
  b = block_sum1(b, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// sc[0] = sum w, sc[1] = fact (np.cov: sw - ddof sw2 / sw, or sw at ddof 0),
// sc[2] = 1 / fact, sc[3] = 1 when sum w > 0 (else the caller reports an error)
__global__ __launch_bounds__(256) void wsum_final(const double* part, int nb, int ddof,
                                                  double* sc) {
  __shared__ double red[4];
  double a = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nb; k += 256) {
    a += part[2 * k];
    b += part[2 * k + 1];
  }
  a = block_sum1(a, red);
  b = block_sum1(b, red);
  if (threadIdx.x == 0) {
    const double fact = ddof == 0 ? a : a - ddof * b / a;
    sc[0] = a;
    sc[1] = fact;
    sc[2] = 1.0 / fact;
    sc[3] = a > 0.0 ? 1.0 : 0.0;
  }
}

// max of lw (one value) for the LOGW weights
__global__ __launch_bounds__(256) void max_part_kernel(const double* x, long long n, double* part) {
  __shared__ double red[4];
  double m = -INFINITY;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    m = fmax(m, x[i]);
  m = block_max1(m, red);
  if (threadIdx.x == 0) part[blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void max_final_kernel(const double* part, int nb, double* out) {
  __shared__ double red[4];
  double m = -INFINITY;
  for (int k = threadIdx.x; k < nb; k += 256) m = fmax(m, part[k]);
  m = block_max1(m, red);
  if (threadIdx.x == 0) *out = m;
}
}  // namespace

size_t bounds_wcov_scratch_doubles(long long n, long long d) {
  return bounds_scratch_doubles(n, d) + (size_t)n * (size_t)d + (size_t)n + 2 * kRedBlocks + 64;
}

// np.average(x.T, axis=1, weights=w) and np.cov(x.T, aweights=w, ddof=ddof) for x
// [n][d], everything on the device: w (raw weights, or log weights with logw:
// exp(lw - max lw)) -> weight sums and np.cov's normaliser in device scalars ->
// weighted column means (row-chunked partials) -> centred weighted products
// (pairwise chunked reduction for d <= kCovDMax, else Xc^T diag(w) Xc on the
// fp64 MFMA GEMM).  w null: the unweighted np.cov with ddof.  sc_out[4] (device)
// receives the scalars (sc_out[3] = 0 when the weights sum to zero).
hipError_t bounds_weighted_covariance(const double* x, long long n, long long d, const double* w,
                                      bool logw, int ddof, double* scratch, double* sc_out,
                                      double* mean, double* cov, hipStream_t s) {
  long long rpc;
  const int nc = col_chunks(n, &rpc);
  double* part = scratch;                                   // reductions
  double* wbuf = scratch + bounds_scratch_doubles(n, d);    // [n] exp weights
  double* xc = wbuf + n;                                    // [n][d] centred x (GEMM path)
  double* red = xc + (size_t)n * d;                         // [2 kRedBlocks + 8]
  const double* wv = w;
  const int g = red_grid(n);
  if (w) {
    if (logw) {
      hipLaunchKernelGGL(max_part_kernel, dim3(g), dim3(256), 0, s, w, n, red);
      hipLaunchKernelGGL(max_final_kernel, dim3(1), dim3(256), 0, s, red, g, red + 2 * kRedBlocks);
      hipLaunchKernelGGL(wsum_kernel<true>, dim3(g), dim3(256), 0, s, w, n,
                         red + 2 * kRedBlocks, wbuf, red);
      wv = wbuf;
    } else {
      hipLaunchKernelGGL(wsum_kernel<false>, dim3(g), dim3(256), 0, s, w, n, nullptr, nullptr, red);
    }
    hipLaunchKernelGGL(wsum_final, dim3(1), dim3(256), 0, s, red, g, ddof, sc_out);
  }
  const double* sw = w ? sc_out : nullptr;
  const double* fact = w ? sc_out + 1 : nullptr;
  hipLaunchKernelGGL(col_sum_kernel, dim3(nc, (unsigned)((d + 63) / 64)), dim3(256), 0, s, x, n, d,
                     rpc, part, wv);
  hipLaunchKernelGGL(col_final_kernel, dim3((unsigned)((d + 255) / 256)), dim3(256), 0, s, part, nc,
                     n, d, mean, sw);
  if (d <= kCovDMax) {
    const int npairs = (int)(d * (d + 1) / 2);
    hipLaunchKernelGGL(cov_kernel, dim3(nc, npairs), dim3(256), 0, s, x, n, d, mean, rpc, part, wv);
    if (!w) {
      // unweighted with ddof: the (n - ddof) normaliser from a device scalar
      hipLaunchKernelGGL(set_scalar_kernel, dim3(1), dim3(1), 0, s, sc_out + 1, (double)(n - ddof));
      fact = sc_out + 1;
    }
    hipLaunchKernelGGL(cov_final_kernel, dim3((npairs + 255) / 256), dim3(256), 0, s, part, nc,
                       npairs, n, d, cov, fact);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(center_kernel, dim3((unsigned)((n * d + 255) / 256)), dim3(256), 0, s, x, n, d,
                     mean, xc);
  GemmOp gm{};
  gm.ta = true;
  gm.tb = false;
  gm.M = (int)d;
  gm.N = (int)d;
  gm.K = (int)n;
  gm.A = xc;
  gm.lda = d;
  gm.B = xc;
  gm.ldb = d;
  gm.C = cov;
  gm.ldc = d;
  gm.alpha = w ? 1.0 : 1.0 / (double)(n - ddof);
  gm.alpha_dev = w ? sc_out + 2 : nullptr;
  gm.kscale = wv;
  hipError_t e = gemm(gm, s);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t bounds_covariance(const double* x, long long n, long long d, double* scratch,
                             double* mean, double* cov, hipStream_t s) {
  hipError_t e = means(x, n, d, scratch, mean, s);
  if (e != hipSuccess) return e;
  long long rpc;
  const int nc = col_chunks(n, &rpc);
  const int npairs = (int)(d * (d + 1) / 2);
  hipLaunchKernelGGL(cov_kernel, dim3(nc, npairs), dim3(256), 0, s, x, n, d, mean, rpc, scratch);
  hipLaunchKernelGGL(cov_final_kernel, dim3((npairs + 255) / 256), dim3(256), 0, s, scratch, nc,
                     npairs, n, d, cov);
  return hipGetLastError();
}

}  // namespace vbk

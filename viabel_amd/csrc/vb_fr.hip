// vb_fr.hip — full-rank Student-t family on the device
// (t_variational_family, viabel/vb.py:192-233; multivariate_t_logpdf,
// viabel/_distributions.py:8-38) and its KLVI / CHIVI value + gradient
// (vb.py:236-266).
//
// lambda = [mu (D), tril(M) row-major (D(D+1)/2)], L = M with exp'd diagonal,
// Sigma = L L^T (paragami PSDSymmetricMatrixPattern).
//
// One step, GEMMs only (fp64 MFMA, vb_gemm.hpp), no eigendecomposition:
//   L <- unpack(lambda);  Sigma <- L L^T;  0.5 log det Sigma = sum log L_ii
//   S = sqrtm(Sigma) by scaled coupled Newton-Schulz on Sigma / c (fr_sqrt)
//   X = mu + (Z S) / s                           (vb.py:208, fused epilogue)
//   G = d log p / dx, log p                      (corr_gauss: G = -X P*, GEMM)
//   KLVI : r_n = -1/N,            c = -1/2       (entropy .5 log det Sigma)
//   CHIVI: r_n = alpha w_n / N,   c = +1/2 sum r (log q's -.5 log det Sigma; the
//          Mahalanobis term is invariant under the reparameterisation)
//   G_S = Z^T diag(r / s) G                       (cotangent of S)
//   autograd's sqrtm VJP solves S X + X S = G_S (solve_sylvester); Sigma = L L^T
//   only needs the symmetric part, so X_sym solves S X + X S = G_S + G_S^T, by
//   preconditioned conjugate gradients (fr_pcg).  H = X_sym + 2 c Sigma^-1;
//   G_L = H L;  grad = [sum r G, tril(G_L) with the diagonal times L_ii], where
//   the Sigma^-1 term reduces to 2 c on the packed log-diagonal.
// No host synchronisation inside a step: scalars (scales, step sizes,
// convergence flags) live on the device (FrSched); fr_info reads the status.
// The eigendecomposition (rocSOLVER dsyevd) remains only for log q of arbitrary
// points (multivariate_t_logpdf's pinv cutoff) and the eigenvalues of
// mean_and_cov / pth_moment, off the optimisation loop.
#include "vb_device.hpp"
#include "vb_internal.hpp"
#include "vb_symsum.hpp"

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <new>

namespace vbk {
using namespace vbd;

namespace {

GemmOp mm(int M, int N, int K, const double* A, bool ta, const double* B, bool tb, double* C,
          double alpha = 1.0) {
  GemmOp g{};
  g.ta = ta;
  g.tb = tb;
  g.M = M;
  g.N = N;
  g.K = K;
  g.A = A;
  g.lda = ta ? M : K;
  g.B = B;
  g.ldb = tb ? K : N;
  g.C = C;
  g.ldc = N;
  g.alpha = alpha;
  g.beta = 0.0;
  return g;
}

inline unsigned blocks(long long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

// ---- elementwise / reduction kernels ------------------------------------------
__global__ __launch_bounds__(256) void fr_unpack_kernel(int D, const double* lam, double* L) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)D * D) return;
  const int i = (int)(idx / D), j = (int)(idx % D);
  const long long base = D + (long long)i * (i + 1) / 2;
  double v = 0.0;
  if (j < i) v = lam[base + j];
  else if (j == i) v = exp(lam[base + i]);
  L[idx] = v;
}

// Block-wide sum / max over 1024 threads.
__device__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double t = 0.0;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) t += red[k];
  return t;
}

__device__ double block_max(double v, double* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double t = red[0];
  const int nw = blockDim.x >> 6;
  for (int k = 1; k < nw; ++k) t = fmax(t, red[k]);
  return t;
}

// scal[0] = 0.5 * sum log w  (= entropy .5 log det Sigma, vb.py:213)
__global__ __launch_bounds__(1024) void fr_logdet_kernel(int D, const double* w, double* scal) {
  __shared__ double red[16];
  double a = 0.0;
  for (int k = threadIdx.x; k < D; k += blockDim.x) a += log(w[k]);
  a = block_sum(a, red);
  if (threadIdx.x == 0) scal[0] = 0.5 * a;
}

// Philox draws: z[n][d] standard normals (column pair d/2, sample n, purpose 0);
// s[n] = sqrt(chisquare(df) / df) = sqrt(2 Gamma(df/2) / df) from the reserved
// column pair 0xFFFFFFFF (vb.py:204-206 draw order has no counterpart here).
__global__ __launch_bounds__(256) void fr_noise_kernel(int D, long long n, Rng rng, uint32_t step,
                                                       double df, double* z, double* s) {
  const int np = (D + 1) / 2;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * (np + 1)) return;
  const long long r = idx / (np + 1);
  const int j = (int)(idx % (np + 1));
  if (j == np) {
    double ga, gb;
    gamma_pair(rng, 0xFFFFFFFFu, (uint32_t)r, step, 0.5 * df, ga, gb);
    s[r] = sqrt(2.0 * ga / df);
    return;
  }
  double z0, z1;
  normal_pair(rng.draw((uint32_t)j, (uint32_t)r, step, 0u), z0, z1);
  z[r * D + 2 * j] = z0;
  if (2 * j + 1 < D) z[r * D + 2 * j + 1] = z1;
}

// The same draws as fr_noise_kernel, one 256-thread block per row n, which also
// reduces zz[n] = sum_d z_nd^2 (the Mahalanobis invariant of log q): the fused
// step needs no separate row pass over z.
__device__ void fr_noise_row(int D, long long r, const Rng& rng, uint32_t step, double df, double* z,
                             double* s, double* zz, double* red) {
  const int np = (D + 1) / 2;
  double a = 0.0;
  for (int j = threadIdx.x; j <= np; j += blockDim.x) {
    if (j == np) {
      double ga, gb;
      gamma_pair(rng, 0xFFFFFFFFu, (uint32_t)r, step, 0.5 * df, ga, gb);
      s[r] = sqrt(2.0 * ga / df);
      continue;
    }
    double z0, z1;
    normal_pair(rng.draw((uint32_t)j, (uint32_t)r, step, 0u), z0, z1);
    z[r * D + 2 * j] = z0;
    a = fma(z0, z0, a);
    if (2 * j + 1 < D) {
      z[r * D + 2 * j + 1] = z1;
      a = fma(z1, z1, a);
    }
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) zz[r] = a;
}

__global__ __launch_bounds__(256) void fr_noise_rows_kernel(int D, Rng rng, uint32_t step, double df,
                                                            double* z, double* s, double* zz) {
  __shared__ double red[16];
  fr_noise_row(D, blockIdx.x, rng, step, df, z, s, zz, red);
}

// One wave per row: zz[n] = sum_d z^2 (maha = zz / s^2), and for corr_gauss
// logp[n] = 0.5 sum_d x G + const (G = -P x).
__global__ __launch_bounds__(256) void fr_rows_kernel(int D, long long n, const double* z,
                                                      const double* x, const double* G,
                                                      double lp_const, int quad, double* zz,
                                                      double* logp) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  double a = 0.0, b = 0.0;
  for (int d = lane; d < D; d += 64) {
    if (z) {
      const double v = z[row * D + d];
      a += v * v;
    }
    if (quad) b += x[row * D + d] * G[row * D + d];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    if (zz) zz[row] = a;
    if (quad) logp[row] = 0.5 * b + lp_const;
  }
}

// Objective weights.  scal: [0] half log det, [1] c (Sigma^-1 coefficient).
// KLVI (vb.py:236-245):  value = -(entropy + mean logp), r_n = -1/N.
// CHIVI (vb.py:248-266): lw = logp - logq, w = exp(lw - max)^alpha,
//   value = log(mean w)/alpha + max, r_n = alpha w_n / N.
// lp_part (fused step, corr_gauss): logp[n] = 0.5 sum_t lp_part[t][n] + lp_const
// from the target GEMM's per-row partials of x . G (n_lp parts), written here.
__global__ __launch_bounds__(1024) void fr_weights_kernel(int N, int D, int chivi, int pd,
                                                          double alpha,
                                                          double df, double t_const,
                                                          double* logp, const double* zz,
                                                          const double* s, double* scal,
                                                          double* r, double* rk, double* value,
                                                          const double* lp_part = nullptr,
                                                          int n_lp = 0, double lp_const = 0.0) {
  __shared__ double red[16];
  if (lp_part) {
    // 8 threads per row (independent loads of every 8th partial), fixed xor tree
    const int T = blockDim.x;
    for (int base = 0; base < N; base += T / 8) {
      const int k = base + (int)threadIdx.x / 8, sub = threadIdx.x & 7;
      double a = 0.0;
      if (k < N) {
#pragma unroll 4
        for (int t = sub; t < n_lp; t += 8) a += lp_part[(long long)t * N + k];
      }
      a += __shfl_xor(a, 1, 64);
      a += __shfl_xor(a, 2, 64);
      a += __shfl_xor(a, 4, 64);
      if (sub == 0 && k < N) logp[k] = 0.5 * a + lp_const;
    }
    __syncthreads();   // logp rows are re-read below by other threads
  }
  const double hld = scal[0];
  const double e = 0.5 * (df + D);
  if (!chivi) {
    double a = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      if (pd) {  // black_box_klvi_pd: log p - log q(x), the Mahalanobis invariant
        const double maha = zz[k] / (s[k] * s[k]);
        a += logp[k] - ((t_const - hld) - e * log(1.0 + maha / df));
      } else {
        a += logp[k];
      }
      r[k] = -1.0 / N;
      rk[k] = (-1.0 / N) / s[k];
    }
    a = block_sum(a, red);
    if (threadIdx.x == 0) {
      *value = pd ? -(a / N) : -(hld + a / N);
      scal[1] = -0.5;
    }
    return;
  }
  double mx = -INFINITY;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    const double maha = zz[k] / (s[k] * s[k]);
    const double logq = (t_const - hld) - e * log(1.0 + maha / df);
    const double lw = logp[k] - logq;
    r[k] = lw;
    mx = fmax(mx, lw);
  }
  mx = block_max(mx, red);
  double sw = 0.0;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    const double w = pow(exp(r[k] - mx), alpha);
    sw += w;
    const double rr = alpha * w / N;
    r[k] = rr;
    rk[k] = rr / s[k];
  }
  sw = block_sum(sw, red);
  if (threadIdx.x == 0) {
    *value = log(sw / N) / alpha + mx;
    scal[1] = 0.5 * alpha * sw / N;
  }
}

// gmu[j] = sum_n r_n G[n][j]: 64 columns per block, the 16 waves take every
// 16th row, fixed-order combine in LDS
__global__ __launch_bounds__(1024) void fr_colsum_kernel(int N, int D, const double* r,
                                                         const double* G, double* out) {
  __shared__ double part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  double a = 0.0;
  if (j < D)
    for (int n = wv; n < N; n += 16) a += r[n] * G[(long long)n * D + j];
  part[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && j < D) {
    double t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      t[q] = (part[4 * q][lane] + part[4 * q + 1][lane]) + (part[4 * q + 2][lane] + part[4 * q + 3][lane]);
    out[j] = (t[0] + t[1]) + (t[2] + t[3]);
  }
}

// grad[D + i(i+1)/2 + j] = G_L[i][j] (j < i), G_L[i][i] L[i][i] + 2 scal[1] (exp on
// the diagonal; the log det term, see fr_value_grad).  Thread 0 also folds this
// step's Newton-Schulz / PCG outcome into the sticky status (FrSched).
template <class Sched>
__global__ __launch_bounds__(256) void fr_pack_kernel(int D, const double* GL, const double* L,
                                                      const double* scal, Sched* sc,
                                                      const double* rr_part, int n_rr,
                                                      double* grad, double pcg_tol2 = 0.0,
                                                      int pcg_last = -1) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0) {
    __shared__ double red[16];
    double rr = 0.0;
    for (int k = threadIdx.x; k < n_rr; k += 256) rr += rr_part[k];
    rr = block_sum(rr, red);
    if (threadIdx.x == 0 && !sc->pcg_done) {
      if (!(rr <= 1e-14 * sc->ee)) sc->status |= 2;  // relative residual above 1e-7
      // the last launched iteration converged: no later launch tested it (the
      // symmetric-sum loop tests R_i at the start of iteration i)
      if (rr <= pcg_tol2 * sc->ee) sc->pcg_iter = pcg_last;
    }
  }
  if (idx == 0) {
    if (!sc->ns_conv && !sc->ns_fin) sc->status |= 1;
    if (sc->warm_step) {
      sc->hint_ns = max(sc->hint_ns, sc->ns_iter);
      sc->hint_pcg = max(sc->hint_pcg, sc->pcg_iter);
      // launches a root needs: through the final update (fin: ns_iter - 1) or
      // through the detecting one (ns_iter)
      if (sc->ns_fin) sc->hint_fin = max(sc->hint_fin, sc->ns_iter - 1);
      else sc->hint_det = max(sc->hint_det, sc->ns_iter);
    }
  }
  if (idx >= (long long)D * D) return;
  const int i = (int)(idx / D), j = (int)(idx % D);
  if (j > i) return;
  double v = GL[idx];
  if (j == i) v = fma(v, L[idx], 2.0 * scal[1]);
  grad[D + (long long)i * (i + 1) / 2 + j] = v;
}

// x - mu, for log q of arbitrary points
__global__ __launch_bounds__(256) void fr_center_kernel(int D, long long n, const double* x,
                                                        const double* mu, double* out) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * D) return;
  out[idx] = x[idx] - mu[idx % D];
}

// multivariate_t_logpdf (_distributions.py:27-37) from Y = (x - mu) V:
// maha = sum_k Y_k^2 * pinv(w_k) with the absolute 1e-10 cutoff.
__global__ __launch_bounds__(256) void fr_logq_kernel(int D, long long n, const double* Y,
                                                      const double* w, const double* scal,
                                                      double df, double t_const, double* out) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  double a = 0.0;
  for (int k = lane; k < D; k += 64) {
    const double wk = w[k];
    const double ip = fabs(wk) <= 1e-10 ? 0.0 : 1.0 / wk;
    const double y = Y[row * D + k] * sqrt(ip);
    a += y * y;
  }
  a = wave_sum(a);
  if (lane == 0) out[row] = (t_const - scal[0]) - 0.5 * (df + D) * log(1.0 + a / df);
}

// *out = ||X - shift I||_F^2 for an n x n X.  Per-block partials; the last block
// to finish (self-resetting ticket) sums them in block order: deterministic.
constexpr int kNormBlocks = 128;
__global__ __launch_bounds__(256) void fr_frob2_kernel(int n, const double* X, double shift,
                                                       double* partial, unsigned* ticket,
                                                       double* out) {
  __shared__ double red[16];
  __shared__ bool last;
  const long long nn = (long long)n * n;
  double a = 0.0;
  for (long long idx = (long long)blockIdx.x * 256 + threadIdx.x; idx < nn;
       idx += 256LL * gridDim.x) {
    double v = X[idx];
    if (idx % (n + 1) == 0) v -= shift;
    a += v * v;
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = a;
    __threadfence();
    last = atomicInc(ticket, gridDim.x - 1) == gridDim.x - 1;
  }
  __syncthreads();
  if (last) {
    __threadfence();
    __shared__ double ps[kNormBlocks];
    for (unsigned b = threadIdx.x; b < gridDim.x; b += 256)
      ps[b] = __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (unsigned b = 0; b < gridDim.x; ++b) t += ps[b];  // fixed order
      *out = t;
    }
  }
}

// Power iteration for lambda_max(Sigma): y = Sigma x / ||x||, 8 rows per block
// (two per wave).  x0 = ones.
__global__ __launch_bounds__(256) void fr_power_kernel(int D, const double* Sig, const double* x,
                                                       double* y) {
  __shared__ double red[16];
  __shared__ double inv_n;
  double a = 0.0;
  for (int i = threadIdx.x; i < D; i += 256) {
    const double v = x ? x[i] : 1.0;
    a += v * v;
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) inv_n = 1.0 / sqrt(a);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int rr = 0; rr < 2; ++rr) {
    const int row = blockIdx.x * 8 + wv * 2 + rr;
    if (row >= D) break;
    double t = 0.0;
    for (int j = lane; j < D; j += 64) t += Sig[(long long)row * D + j] * (x ? x[j] : 1.0);
    t = wave_sum(t);
    if (lane == 0) y[row] = t * inv_n;
  }
}

// *out = ||x||^2 (one block)
__global__ __launch_bounds__(256) void fr_norm2_kernel(int n, const double* x, double* out) {
  __shared__ double red[16];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) a += x[i] * x[i];
  a = block_sum(a, red);
  if (threadIdx.x == 0) *out = a;
}

// ---- Newton-Schulz schedule (device) -------------------------------------------
// Coupled scaled Newton-Schulz on A = Sigma / c (Higham, Functions of Matrices
// §6.3, with the Chen-Chow scaling): for k >= 0
//   T_k = 3 I - a_k^2 Z_k Y_k,  Y_{k+1} = a_k Y_k T_k / 2,  Z_{k+1} = a_k T_k Z_k / 2,
//   Y_0 = A, Z_0 = I.  Eigenvalue-wise x = sqrt(p), p of Z_k Y_k:
//   x' = a x (3 - a^2 x^2) / 2 with a = sqrt(3 / (1 + l + l^2)) maps [l, 1] into
//   [f(l), 1], so the lower bound l_k of x sets every a_k; a_k -> 1 as l_k -> 1.
//   Y_k -> A^(1/2), Z_k -> A^(-1/2).
// Scalars (FrSched, device): c = min(1.25 x power estimate of lambda_max,
// ||Sigma||_F); l_0 = 0.8 sqrt(lambda_min / c) with lambda_min from the previous
// root (||Z_prev||_2 by power iteration: lambda_min = c_prev / ||Z_prev||^2), or
// l_default without one.  A low l_0 costs iterations, never accuracy: the
// iteration is declared converged from the residual ||I - Z_k Y_k||_F alone.
struct FrSched {
  double c, sqrt_c, inv_sqrt_c;
  double cbuf[2];                // c of the last two roots: a schedule reads the previous
                                 // one at [slot ^ 1] and writes its own at [slot] (the
                                 // fused iteration-0 GEMM's blocks read while block 0 writes)
  double ns0[4];                 // iteration 0 coefficients (GemmOp::ns0)
  double nalpha2[kFrNSMax + 1];  // -a_k^2 (T_k GEMM alpha)
  double shift[kFrNSMax + 1];    // 3 - a_k^2 (residual shift of T_k)
  double halpha[kFrNSMax + 1];   // a_k / 2
  double inv_a4[kFrNSMax + 1];   // 1 / a_k^4 (residual scale)
  double rz[2], ee;              // PCG: <R, M^-1 R> (by iteration parity), ||E||^2
  double l0, lmax_est;
  double ee_scale;               // PCG: (2 / kappa)^2 when the preconditioned condition
                                 // number kappa > 2, else 1 (see fr_sched_kernel)
  int ns_conv, ns_iter, pcg_done, pcg_iter;
  int ns_fin;                    // the last Newton-Schulz update was final (see fr_sqrt)
  int status;                    // sticky: 1 NS not converged, 2 PCG not converged
  int hint_ns, hint_pcg;         // sticky maxima of the iteration counts
  int hint_fin, hint_det;        // sticky maxima of the launches needed (final update /
                                 // detection), see fr_info
  int warm_step;                 // this root was warm-started (its count feeds hint_ns)
};

// y = M x / ||x|| for (Sigma, x) in grid row 0 and (Z_prev, u) in grid row 1
// (8 rows per block, two per wave).  x null: x = ones.
__global__ __launch_bounds__(256) void fr_power2_kernel(int D, const double* Sig, const double* x,
                                                        double* y, const double* Zp,
                                                        const double* u, double* v) {
  __shared__ double red[16];
  __shared__ double inv_n;
  const double* M = blockIdx.y ? Zp : Sig;
  const double* in = blockIdx.y ? u : x;
  double* out = blockIdx.y ? v : y;
  double a = 0.0;
  for (int i = threadIdx.x; i < D; i += 256) {
    const double t = in ? in[i] : 1.0;
    a += t * t;
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) inv_n = 1.0 / sqrt(a);
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int rr = 0; rr < 2; ++rr) {
    const int row = blockIdx.x * 8 + wv * 2 + rr;
    if (row >= D) break;
    double t = 0.0;
    for (int j = lane; j < D; j += 64) t += M[(long long)row * D + j] * (in ? in[j] : 1.0);
    t = wave_sum(t);
    if (lane == 0) out[row] = t * inv_n;
  }
}

// The schedule's scalar math uses hardware reciprocal / reciprocal-sqrt seeds and
// Newton steps (a few dependent FMAs each) instead of IEEE division and sqrt
// (long software sequences): it runs on one thread on the step's critical path,
// and any deterministic value of these scaling coefficients is a valid schedule
// (Newton-Schulz converges to the same root; the fused and stand-alone schedule
// share this code, so they agree bit for bit).
__device__ __forceinline__ double frcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  return r * fma(-x, r, 2.0);
}
__device__ __forceinline__ double frsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * fma(-0.5 * x, y * y, 1.5);
  return y * fma(-0.5 * x, y * y, 1.5);
}
__device__ __forceinline__ double ns_alpha(double l) {
  return 1.7320508075688772 * frsq(1.0 + l + l * l);   // sqrt(3 / (1 + l + l^2))
}

// The schedule from the reduced sums (f = ||Sigma||_F^2 partial sum, ly / lv =
// ||y||^2 / ||v||^2, ld = sum log L_ii, qf = y^T Sigma y): one thread computes
// c, l_0 and the iteration-0 coefficients ns0[4]; with `a` non-null also the
// per-iteration a_k (k <= kmax) into a[] and the scalar fields of FrSched
// (write), for fr_schedule_store to spread over threads.
__device__ void fr_schedule(int kmax, double f, double ly, double lv, double ld, double qf,
                            bool has_qf, int has_z, double l_default, FrSched* sc, int slot,
                            double* scal, bool write, double* ns0, double* a_out) {
  const double lmax = has_qf ? (ly > 0.0 ? qf * frcp(ly) : 0.0) : ly * frsq(ly);
  const double c = fmin(1.25 * lmax, f * frsq(f));   // ||Sigma||_F >= lambda_max
  const double ic = frcp(c);
  double l = l_default;
  double ee_scale = 1.0;
  if (has_z && lv > 0.0) {
    const double lmin = sc->cbuf[slot ^ 1] * frcp(lv);   // lambda_min(Sigma_prev)
    const double q = lmin * ic;
    l = 0.8 * q * frsq(q);
    // the PCG's X carries up to kappa x its relative residual, kappa = (2 + k +
    // 1/k) / 4 the preconditioned condition number, k = cond(S) = sqrt(lmax /
    // lmin): past kappa = 2 the stopping test tightens by kappa / 2, so X's
    // relative error stays <= 2 x the tolerance however ill-conditioned Sigma is
    // (config 4: kappa ~1.2, unchanged)
    if (write && lmin > 0.0 && lmax > lmin) {
      const double r = lmax * frcp(lmin), k = r * frsq(r), kap = 0.25 * (2.0 + k + frcp(k));
      if (kap > 2.0) ee_scale = 4.0 * frcp(kap * kap);
    }
  }
  l = fmin(fmax(l, 1e-4), 1.0);
  {
    const double a = ns_alpha(l), a2 = a * a;
    // Y_1 = (3/2) a A - (1/2) a^3 A^2, Z_1 = (a / 2) (3 I - a^2 A), A = Sigma / c
    ns0[0] = -0.5 * a * a2 * (ic * ic);
    ns0[1] = 1.5 * a * ic;
    ns0[2] = 0.5 * a;
    ns0[3] = a2 * ic;
  }
  if (!write) return;
  scal[0] = ld;
  sc->ee_scale = ee_scale;
  sc->l0 = l;
  sc->lmax_est = lmax;
  sc->c = c;
  const double rc = frsq(c);
  sc->sqrt_c = c * rc;
  sc->inv_sqrt_c = rc;
  sc->cbuf[slot] = c;
  for (int k = 0; k < 4; ++k) sc->ns0[k] = ns0[k];
  const int kn = kmax < kFrNSMax ? kmax : kFrNSMax;
  for (int k = 0; k <= kn; ++k) {
    const double a = ns_alpha(l), a2 = a * a;
    a_out[k] = a;
    l = fmin(0.5 * a * l * (3.0 - a2 * l * l), 1.0);
  }
  sc->ns_conv = 0;
  sc->ns_fin = 0;
  sc->ns_iter = -1;
  sc->warm_step = has_z;
  sc->pcg_done = 0;
  sc->pcg_iter = -1;
}

// per-iteration coefficients from a_k, one k per thread (after fr_schedule)
__device__ __forceinline__ void fr_schedule_store(int kmax, const double* a_k, FrSched* sc) {
  const int k = threadIdx.x;
  if (k <= kmax && k <= kFrNSMax) {
    const double a = a_k[k], a2 = a * a;
    sc->nalpha2[k] = -a2;
    sc->shift[k] = 3.0 - a2;
    sc->halpha[k] = 0.5 * a;
    sc->inv_a4[k] = frcp(a2 * a2);
  }
}

__global__ __launch_bounds__(1024) void fr_sched_kernel(int D, int kmax, const double* fro_part,
                                                       int n_part, const double* y,
                                                       const double* v, int has_z,
                                                       double l_default, FrSched* sc,
                                                       const double* lam, double* scal,
                                                       const double* qf_part, double* uS,
                                                       double* uZ, int slot) {
  __shared__ double red[16];
  const int T = blockDim.x;
  double f = 0.0, ly = 0.0, lv = 0.0, ld = 0.0, qf = 0.0;
  for (int i = threadIdx.x; i < n_part; i += T) {
    f += fro_part[i];
    if (qf_part) qf += qf_part[i];
  }
  for (int i = threadIdx.x; i < D; i += T) {
    ly += y[i] * y[i];
    if (has_z) lv += v[i] * v[i];
    ld += lam[D + (long long)i * (i + 1) / 2 + i];
  }
  f = block_sum(f, red);
  __syncthreads();
  ly = block_sum(ly, red);
  __syncthreads();
  lv = block_sum(lv, red);
  __syncthreads();
  ld = block_sum(ld, red);
  if (qf_part) {
    __syncthreads();
    qf = block_sum(qf, red);
  }
  {
    const double iy = ly > 0.0 ? frsq(ly) : 0.0, iv = lv > 0.0 ? frsq(lv) : 0.0;
    for (int i = threadIdx.x; i < D; i += T) {
      uS[i] = y[i] * iy;
      if (has_z && lv > 0.0) uZ[i] = v[i] * iv;
    }
  }
  __shared__ double a_k[kFrNSMax + 1];
  if (threadIdx.x == 0) {
    double ns0[4];
    fr_schedule(kmax, f, ly, lv, ld, qf, qf_part != nullptr, has_z, l_default, sc, slot, scal,
                true, ns0, a_k);
  }
  __syncthreads();
  fr_schedule_store(kmax, a_k, sc);
}

// fr_sched_kernel's work inside the Newton-Schulz iteration-0 GEMM (whose
// coefficients are the only use of the schedule in that launch): every block
// loads its share of the partial sums before the main loop, reduces them after
// it (the loads' latency hides under the product) and computes the schedule;
// block 0 stores it (FrSched, uS / uZ, scal) for the launches that follow.  For
// D <= kSchedHookMaxD (the per-thread load counts below).
constexpr int kSchedP = 4, kSchedV = 2;   // partials / vector entries per thread
constexpr int kSchedHookMaxD = kSchedV * 512;
struct SchedArgs {
  int D, kmax, n_part, has_z, slot;
  double l_default;
  const double *fro_part, *qf_part, *y, *v, *lam;
  FrSched* sc;
  double *scal, *uS, *uZ;
};
struct SchedHook {
  using Args = SchedArgs;
  static constexpr bool kKScale = false;
  static constexpr int kLds = 128;
  static constexpr int kEpi = kEpiSym | kEpiNs0;   // the iteration-0 product's epilogue
  const SchedArgs& a;
  const int blk;
  double* const lds;
  double fp[kSchedP], qp[kSchedP], yv[kSchedV], vv[kSchedV], dv[kSchedV];
  __device__ __forceinline__ SchedHook(const SchedArgs& args, int b, double* l)
      : a(args), blk(b), lds(l) {}
  __device__ __forceinline__ const double* kscale() const { return nullptr; }
  __device__ __forceinline__ void pre() {
    const int D = a.D, n_part = a.n_part, has_z = a.has_z;
    const double *fro_part = a.fro_part, *qf_part = a.qf_part, *y = a.y, *v = a.v, *lam = a.lam;
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < kSchedP; ++e) {
      const int i = t + 512 * e;
      fp[e] = i < n_part ? fro_part[i] : 0.0;
      qp[e] = (qf_part && i < n_part) ? qf_part[i] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < kSchedV; ++e) {
      const int i = t + 512 * e;
      yv[e] = i < D ? y[i] : 0.0;
      vv[e] = (has_z && i < D) ? v[i] : 0.0;
      dv[e] = i < D ? lam[D + (long long)i * (i + 1) / 2 + i] : 0.0;
    }
  }
  __device__ __forceinline__ const double* post() {
    const int D = a.D, has_z = a.has_z;
    double* uS = a.uS;
    double* uZ = a.uZ;
    double s5[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int e = 0; e < kSchedP; ++e) {
      s5[0] += fp[e];
      s5[4] += qp[e];
    }
#pragma unroll
    for (int e = 0; e < kSchedV; ++e) {
      s5[1] += yv[e] * yv[e];
      s5[2] += vv[e] * vv[e];
      s5[3] += dv[e];
    }
    const int t = threadIdx.x, w = t >> 6;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      s5[k] = wave_sum(s5[k]);
      if ((t & 63) == 0) lds[8 + 5 * w + k] = s5[k];
    }
    __syncthreads();
    if (t == 0) {
      double r[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      for (int ww = 0; ww < 8; ++ww)
        for (int k = 0; k < 5; ++k) r[k] += lds[8 + 5 * ww + k];
      fr_schedule(a.kmax, r[0], r[1], r[2], r[3], r[4], a.qf_part != nullptr, has_z, a.l_default,
                  a.sc, a.slot, a.scal, blk == 0, lds, lds + 64);
      lds[4] = r[1] > 0.0 ? frsq(r[1]) : 0.0;
      lds[5] = r[2] > 0.0 ? frsq(r[2]) : 0.0;
    }
    __syncthreads();
    if (blk == 0) {   // the per-iteration coefficients and the next step's unit power vectors
      fr_schedule_store(a.kmax, lds + 64, a.sc);
      const double iy = lds[4], iv = lds[5];
#pragma unroll
      for (int e = 0; e < kSchedV; ++e) {
        const int i = t + 512 * e;
        if (i < D) {
          uS[i] = yv[e] * iy;
          if (has_z && iv > 0.0) uZ[i] = vv[e] * iv;
        }
      }
    }
    return lds;
  }
};

// fr_weights_kernel's work inside the G_S = Z^T diag(rk) G GEMM, whose only use of
// the weights is the K scale rk: every block forms the N log weights (log p from
// the target GEMM's row partials, log q from zz and s) and the KLVI / CHIVI
// weights itself, in one fixed order, while the first operand stage is in
// flight, and keeps rk in LDS for the K-scaled LDS-DMA loop; block 0 stores
// logp, r, rk, the objective value and scal[1] for the launches that follow.
// N <= 512, N a multiple of the loop's 64-deep stages.
struct WeightsArgs {
  int N, D, chivi, pd;
  double alpha, df, t_const;
  double* logp;
  const double *zz, *s;
  double *scal, *r, *rk, *value;
  const double* lp_part;
  int n_lp;
  double lp_const;
};
struct WeightsHook {
  using Args = WeightsArgs;
  static constexpr bool kKScale = true;
  static constexpr int kLds = 512 + 64;
  static constexpr int kEpi = 0;
  const WeightsArgs& a;
  const int blk;
  double* const lds;
  __device__ __forceinline__ WeightsHook(const WeightsArgs& args, int b, double* l)
      : a(args), blk(b), lds(l) {}
  __device__ __forceinline__ const double* kscale() const { return lds; }
  __device__ __forceinline__ const double* post() { return nullptr; }
  // fixed-order block reduction over 512 threads (8 waves): op 0 sum, 1 max
  __device__ __forceinline__ double reduce(double v, bool mx) {
    double* red = lds + 512;
    const int t = threadIdx.x;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double o = __shfl_xor(v, off, 64);
      v = mx ? fmax(v, o) : v + o;
    }
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    double r = red[0];
    for (int w = 1; w < 8; ++w) r = mx ? fmax(r, red[w]) : r + red[w];
    __syncthreads();
    return r;
  }
  __device__ __forceinline__ void pre() {
    const int N = a.N, t = threadIdx.x;
    const int tpr = N <= 64 ? 8 : N <= 128 ? 4 : N <= 256 ? 2 : 1;   // threads per row
    const int k = t / tpr, sub = t % tpr;
    const bool own = k < N && sub == 0;
    double lp = 0.0;
    if (a.lp_part) {
      double acc = 0.0;
      if (k < N) {
#pragma unroll 4
        for (int j = sub; j < a.n_lp; j += tpr) acc += a.lp_part[(long long)j * N + k];
      }
      for (int off = 1; off < tpr; off <<= 1) acc += __shfl_xor(acc, off, 64);
      lp = 0.5 * acc + a.lp_const;
    } else if (own) {
      lp = a.logp[k];
    }
    const double hld = a.scal[0];
    const double e = 0.5 * (a.df + a.D);
    double sk = 1.0, lw = 0.0;
    if (own) {
      sk = a.s[k];
      if (a.chivi || a.pd) {
        const double maha = a.zz[k] / (sk * sk);
        lw = lp - ((a.t_const - hld) - e * log(1.0 + maha / a.df));
      }
    }
    if (blk == 0 && own && a.lp_part) a.logp[k] = lp;
    if (!a.chivi) {
      const double tot = reduce(own ? (a.pd ? lw : lp) : 0.0, false);
      if (own) {
        lds[k] = (-1.0 / N) / sk;
        if (blk == 0) {
          a.r[k] = -1.0 / N;
          a.rk[k] = lds[k];
        }
      }
      if (blk == 0 && t == 0) {
        *a.value = a.pd ? -(tot / N) : -(hld + tot / N);
        a.scal[1] = -0.5;
      }
    } else {
      const double mx = reduce(own ? lw : -INFINITY, true);
      const double w = own ? pow(exp(lw - mx), a.alpha) : 0.0;
      const double sw = reduce(w, false);
      if (own) {
        const double rr = a.alpha * w / N;
        lds[k] = rr / sk;
        if (blk == 0) {
          a.r[k] = rr;
          a.rk[k] = lds[k];
        }
      }
      if (blk == 0 && t == 0) {
        *a.value = log(sw / N) / a.alpha + mx;
        a.scal[1] = 0.5 * a.alpha * sw / N;
      }
    }
    __syncthreads();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
};

// VIABEL_AMD_FR_WEIGHTS_FUSE=0: the weights kernel runs on its own instead of
// inside the G_S GEMM (WeightsHook; A/B switch: config 4 0.431 -> 0.426 ms/step)
bool weights_fused() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_FR_WEIGHTS_FUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The fused step's last kernel (adagrad runs, Philox draws): the packed gradient
// of fr_pack_kernel goes straight into the windowed adagrad step (adagrad_step,
// as adagrad_update_kernel) and L of the new parameters is written for the next
// step's Sigma GEMM (no unpack); extra blocks prepare the next step: its draws
// (fr_noise_row, with zz) and one power step each on this step's Sigma and root
// Z (pS = Sigma uS, pz = Z uZ).  Blocks [0, npb): parameters (mu first, then the
// packed lower triangle), [npb, npb + nrows): draw rows, then nzb blocks of
// Sigma rows and nzb of Z rows (8 per block).
struct FrPackArgs {
  int D, npb, nrows, nzb;
  const double* GL;
  double* L;
  const double* scal;
  FrSched* sc;
  const double* rr_part;
  int n_rr;
  double pcg_tol2;   // see fr_pack_kernel
  int pcg_last;
  const double* gmu;   // mean gradient (pcg_init's colsum blocks)
  double* lam;
  double* ring;
  int W;
  long long step;
  double lr, eps;
  double* hrow;
  // next step
  Rng rng;
  uint32_t next_step;
  double df;
  double *z, *s, *zz;
  const double *Zf, *uZ, *Sig, *uS;
  double *pz, *pS;
};

__global__ __launch_bounds__(256) void fr_pack_update_kernel(FrPackArgs a) {
#ifndef VB_NO_KWARM
  kernarg_warm(a);
#endif
  __shared__ double red[16];
  const int D = a.D;
  const int b = blockIdx.x;
  if (b >= a.npb) {
    const int k = b - a.npb;
    if (k < a.nrows) {
      fr_noise_row(D, k, a.rng, a.next_step, a.df, a.z, a.s, a.zz, red);
      return;
    }
    // power steps pS = Sigma uS (blocks [0, nzb)) and pz = Z uZ (the next nzb):
    // two rows per wave
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int zb = k - a.nrows;
    const bool zside = zb >= a.nzb;
    if (zside) zb -= a.nzb;
    const double* M = zside ? a.Zf : a.Sig;
    const double* u = zside ? a.uZ : a.uS;
    double* out = zside ? a.pz : a.pS;
    for (int rr = 0; rr < 2; ++rr) {
      const int row = zb * 8 + wv * 2 + rr;
      if (row >= D) break;
      double t = 0.0;
      for (int j = lane; j < D; j += 64) t = fma(M[(long long)row * D + j], u[j], t);
      t = wave_sum(t);
      if (lane == 0) out[row] = t;
    }
    return;
  }
  const long long p = (long long)b * 256 + threadIdx.x;
  if (b == 0) {
    // the last PCG residual, summed by the whole block (one thread's serial loop
    // over the partials took ~20 us)
    double rr = 0.0;
    for (int k = threadIdx.x; k < a.n_rr; k += 256) rr += a.rr_part[k];
    rr = block_sum(rr, red);
    FrSched* sc = a.sc;
    if (threadIdx.x == 0 && !sc->pcg_done) {
      if (!(rr <= 1e-14 * sc->ee)) sc->status |= 2;  // relative residual above 1e-7
      if (rr <= a.pcg_tol2 * sc->ee) sc->pcg_iter = a.pcg_last;
    }
  }
  if (p == 0) {
    FrSched* sc = a.sc;
    if (!sc->ns_conv && !sc->ns_fin) sc->status |= 1;
    if (sc->warm_step) {
      sc->hint_ns = max(sc->hint_ns, sc->ns_iter);
      sc->hint_pcg = max(sc->hint_pcg, sc->pcg_iter);
      // launches a root needs: through the final update (fin: ns_iter - 1) or
      // through the detecting one (ns_iter)
      if (sc->ns_fin) sc->hint_fin = max(sc->hint_fin, sc->ns_iter - 1);
      else sc->hint_det = max(sc->hint_det, sc->ns_iter);
    }
  }
  const long long P = D + (long long)D * (D + 1) / 2;
  if (p >= P) return;
  double g;
  long long li = -1;
  bool diag = false;
  if (p < D) {
    g = a.gmu[p];
  } else {
    const long long k = p - D;
    long long i = (long long)((sqrt(8.0 * (double)k + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= k) ++i;
    while (i * (i + 1) / 2 > k) --i;
    const long long j = k - i * (i + 1) / 2;
    li = i * D + j;
    diag = i == j;
    g = a.GL[li];
    if (diag) g = fma(g, a.L[li], 2.0 * a.scal[1]);
  }
  const double v = adagrad_step(p, P, a.lam[p], g, a.ring, a.W, a.step, a.lr, a.eps, nullptr);
  a.lam[p] = v;
  if (a.hrow) a.hrow[p] = v;
  if (li >= 0) a.L[li] = diag ? exp(v) : v;
}

// ---- PCG for the sqrtm VJP ----------------------------------------------------
// autograd's sqrtm VJP solves S X + X S = G_S (solve_sylvester); Sigma = L L^T
// needs only the symmetric part: S X + X S = E, E = G_S + G_S^T.  In the scaled
// variables Y = A^(1/2) = S / sqrt(c), Z = Y^-1: Y X + X Y = E / sqrt(c) =: Eh.
// The operator L(X) = Y X + X Y is SPD on symmetric matrices (Frobenius inner
// product); the preconditioner M^-1(R) = (Z R + R Z) / 4 has eigenvalues
// (1/4)(1/y_i + 1/y_j) against L's (y_i + y_j), so the preconditioned spectrum
// lies in [1, (2 + k + 1/k) / 4] for k = cond(Y) (1.17 at config 4): conjugate
// gradients reach 1e-11 in ~7 iterations, two GEMMs each (Y P and Z R; the
// transposes of the symmetric products are read by the update kernels).
// Inner products ride in GEMM epilogues (<P, Y P> = <P, L(P)> / 2, <R, Z R> =
// 2 <R, M^-1 R>) and in the update kernels, as per-block partials that every
// consumer block sums in the same order (no atomics).
constexpr int kTile = 32;

// 32 x 32 tile (bi, bj) of M and of M^T through LDS: thread t owns 4 elements.
struct TileT {
  __device__ static void load_t(const double* M, int D, int bi, int bj, double (*s)[kTile + 1]) {
    for (int e = threadIdx.x; e < kTile * kTile; e += 256) {
      const int r = e / kTile, cc = e % kTile;
      const int gr = bj * kTile + r, gc = bi * kTile + cc;
      s[r][cc] = (gr < D && gc < D) ? M[(long long)gr * D + gc] : 0.0;
    }
    __syncthreads();
  }
};

// Sum of n per-block partials by the whole (256-thread) block, in a fixed
// order: every block of a grid gets the bitwise-identical total.
__device__ double sum_parts(const double* p, int n, double* red) {
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) a += p[i];
  return block_sum(a, red);
}

// gmu[j] = sum_n r_n Gm[n][j] by one 256-thread block per 64 columns (the
// fused step's mean gradient, run as extra blocks of pcg_init_kernel): 4 waves
// take every 4th row, combined in a fixed order
__device__ void colsum_block(int N, int D, int cb, const double* r, const double* Gm, double* gmu) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = cb * 64 + lane;
  double a = 0.0;
  if (j < D) {
#pragma unroll 8
    for (int n = wv; n < N; n += 4) a = fma(r[n], Gm[(long long)n * D + j], a);
  }
  part[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && j < D) gmu[j] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}

// Eh = (G + G^T) / sqrt(c), R = Eh, X = 0, ee partials.  Blocks of the extra grid
// row blockIdx.y == gridDim.x (when n_cs > 0) compute the mean gradient instead.
__global__ __launch_bounds__(256) void pcg_init_kernel(int D, const double* G, const FrSched* sc,
                                                       double* Eh, double* R, double* X,
                                                       double* ee_part, int n_cs = 0, int N = 0,
                                                       const double* rw = nullptr,
                                                       const double* Gm = nullptr,
                                                       double* gmu = nullptr) {
  __shared__ double s[kTile][kTile + 1];
  __shared__ double red[16];
  if ((int)blockIdx.y == (int)gridDim.x) {
    if ((int)blockIdx.x < n_cs) colsum_block(N, D, blockIdx.x, rw, Gm, gmu);
    return;
  }
  const int bi = blockIdx.y, bj = blockIdx.x;
  TileT::load_t(G, D, bi, bj, s);
  const double isc = sc->inv_sqrt_c;
  double a = 0.0;
  for (int e = threadIdx.x; e < kTile * kTile; e += 256) {
    const int r = e / kTile, cc = e % kTile;
    const int i = bi * kTile + r, j = bj * kTile + cc;
    if (i < D && j < D) {
      const long long idx = (long long)i * D + j;
      const double v = (G[idx] + s[cc][r]) * isc;
      Eh[idx] = v;
      R[idx] = v;
      X[idx] = 0.0;
      a += v * v;
    }
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) ee_part[blockIdx.y * gridDim.x + blockIdx.x] = a;
}

// The update kernels below issue every global load of the block (their tile of
// C^T for the LDS transpose, their own elements, the partials) before the first
// barrier, so the load latencies overlap instead of adding up; the partials are
// summed in the same per-thread order as sum_parts (bitwise-identical totals).
constexpr int kPer = kTile * kTile / 256;   // elements per thread

// X += alpha P, R -= alpha (C + C^T), rr partials;  alpha = rz / <P, L(P)>,
// <P, L(P)> = 2 sum(pq_part)
__global__ __launch_bounds__(256) void pcg_xr_kernel(int D, int it, const double* C,
                                                     const double* P, const double* pq_part,
                                                     int n_pq, FrSched* sc, double* X, double* R,
                                                     double* rr_part) {
  __shared__ double s[kTile][kTile + 1];
  __shared__ double red[16];
  if (sc->pcg_done) return;
  const int bi = blockIdx.y, bj = blockIdx.x;
  double ct[kPer], cv[kPer], pv[kPer], xv[kPer], rv[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e, r = q / kTile, cc = q % kTile;
    const int tr = bj * kTile + r, tc = bi * kTile + cc;     // transposed tile element
    ct[e] = (tr < D && tc < D) ? C[(long long)tr * D + tc] : 0.0;
    const int i = bi * kTile + r, j = bj * kTile + cc;
    const bool ok = i < D && j < D;
    const long long idx = (long long)i * D + j;
    cv[e] = ok ? C[idx] : 0.0;
    pv[e] = ok ? P[idx] : 0.0;
    xv[e] = ok ? X[idx] : 0.0;
    rv[e] = ok ? R[idx] : 0.0;
  }
  double pq = 0.0;
  for (int k = threadIdx.x; k < n_pq; k += 256) pq += pq_part[k];
  const double rz = sc->rz[it & 1];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e;
    s[q / kTile][q % kTile] = ct[e];
  }
  const double alpha = rz / (2.0 * block_sum(pq, red));   // barriers: s is complete
  double a = 0.0;
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e, r = q / kTile, cc = q % kTile;
    const int i = bi * kTile + r, j = bj * kTile + cc;
    if (i < D && j < D) {
      const long long idx = (long long)i * D + j;
      X[idx] = fma(alpha, pv[e], xv[e]);
      const double rn = rv[e] - alpha * (cv[e] + s[cc][r]);
      R[idx] = rn;
      a += rn * rn;
    }
  }
  a = block_sum(a, red);
  if (threadIdx.x == 0) rr_part[blockIdx.y * gridDim.x + blockIdx.x] = a;
}

// P = (C + C^T) / 4 + beta P with <R, M^-1 R> = sum(rz_part) / 2 and
// beta = <R, M^-1 R> / rz_prev (it < 0: the initial P, beta = 0; block 0 also
// stores ||E||^2).  Block 0 records the new rz for the next iteration.
__global__ __launch_bounds__(256) void pcg_p_kernel(int D, int it, const double* C,
                                                    const double* rz_part, int n_rz,
                                                    const double* ee_part, int n_ee, FrSched* sc,
                                                    double* P) {
  __shared__ double s[kTile][kTile + 1];
  __shared__ double red[16];
  if (sc->pcg_done) return;
  const int bi = blockIdx.y, bj = blockIdx.x;
  double ct[kPer], cv[kPer], pv[kPer];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e, r = q / kTile, cc = q % kTile;
    const int tr = bj * kTile + r, tc = bi * kTile + cc;
    ct[e] = (tr < D && tc < D) ? C[(long long)tr * D + tc] : 0.0;
    const int i = bi * kTile + r, j = bj * kTile + cc;
    const bool ok = i < D && j < D;
    const long long idx = (long long)i * D + j;
    cv[e] = ok ? C[idx] : 0.0;
    pv[e] = (ok && it >= 0) ? P[idx] : 0.0;
  }
  double rzp = 0.0, eep = 0.0;
  for (int k = threadIdx.x; k < n_rz; k += 256) rzp += rz_part[k];
  if (it < 0)
    for (int k = threadIdx.x; k < n_ee; k += 256) eep += ee_part[k];
  const double rz_prev = it < 0 ? 1.0 : sc->rz[it & 1];
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e;
    s[q / kTile][q % kTile] = ct[e];
  }
  const double rz = 0.5 * block_sum(rzp, red);   // barriers: s is complete
  const double beta = it < 0 ? 0.0 : rz / rz_prev;
  double ee = 0.0;
  if (it < 0) {
    __syncthreads();
    ee = block_sum(eep, red);
  }
#pragma unroll
  for (int e = 0; e < kPer; ++e) {
    const int q = threadIdx.x + 256 * e, r = q / kTile, cc = q % kTile;
    const int i = bi * kTile + r, j = bj * kTile + cc;
    if (i < D && j < D) {
      const double z = 0.25 * (cv[e] + s[cc][r]);
      P[(long long)i * D + j] = it < 0 ? z : fma(beta, pv[e], z);
    }
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    sc->rz[(it + 1) & 1] = rz;
    if (it < 0) sc->ee = ee * sc->ee_scale;
  }
}

// ---- PCG on symmetric-sum products (D % 64 == 0; vb_symsum.hpp) --------------
// The same preconditioned CG as above (operator L(P) = Y P + P Y, preconditioner
// M^-1(R) = (Z R + R Z) / 4, X_0 = 0, R_0 = Eh), with the preconditioned residual
// carried by a recurrence instead of recomputed:
//   A_i:  W = L(U_i);  beta = gamma_i / gamma_{i-1} (0 at i = 0);
//         P_i = U_i + beta P_{i-1};  Q_i = W + beta Q_{i-1}  (= L(P_i));  pi_i = <P_i, Q_i>
//   M_i:  V = M^-1(Q_i);  alpha = gamma_i / pi_i;
//         X += alpha P_i;  R -= alpha Q_i;  U -= alpha V  (= M^-1(R));  gamma_{i+1} = <R, U>
// Every update of launch k needs only whole entries of its own product (each block
// owns complete entries of the symmetric result) and scalars summed from the
// partials of launch k - 1, so the vector updates run in the products' epilogues:
// two launches per iteration instead of two products and two update kernels.  In
// exact arithmetic the iterates are the standard loop's.
// Modes: 0 = M^-1(R_0) (U_0, gamma_0; block 0 stores ||E||^2), 1 = A_i, 2 = M_i.
struct SsPcgArgs {
  int D, mode, it;
  const double* Mat;     // Z (modes 0, 2) or Y (mode 1)
  const double* V;       // the product's CG operand: R (0), U (1), Q (2)
  double *R, *U, *P, *Q, *X;
  const double* ee_part;
  int n_ee;
  double* gam;           // [2][nblk]: gamma partials by iteration parity
  double* pi;            // [nblk]
  double* rho;           // [nblk]: ||R||^2 partials (convergence, status)
  FrSched* sc;
  double tol2;           // converged when ||R||^2 <= tol2 ||E||^2 (ee)
  int pcg_call;          // (VB_SS_PROF: index of the PCG call in the workspace's life)
};

// Partials of earlier launches, loaded before a product and summed after it by
// every wave on its own (no block barrier; every wave of every block forms the
// same total in the same order): lane l holds partials l + 64 k (k < 4) as plain
// loads at clamped indices, their validity applied at the sum (a select or a loop
// around a load made the compiler wait for it at once, before the product);
// partials past 256 (D > 512) load at the sum.
struct PartLoad {
  double v[4];
  __device__ __forceinline__ void load(const double* p, int n) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[l + 64 * k < n ? l + 64 * k : 0];
  }
  __device__ __forceinline__ double total(const double* p, int n) const {
    const int l = threadIdx.x & 63;
    double a = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) a += l + 64 * k < n ? v[k] : 0.0;
    for (int i = l + 256; i < n; i += 64) a += p[i];
    return vbd::wave_sum_dpp(a);
  }
};

template <int KT>
__global__ __launch_bounds__(symsum::NTH) void fr_pcg_ss_kernel(SsPcgArgs a) {
  using namespace symsum;
  extern __shared__ double lds[];
  __shared__ double scr[24];
#ifdef VB_SS_PROF
  const unsigned long long p_entry = __builtin_amdgcn_s_memrealtime();
#endif
  kernarg_warm(a);
  asm volatile("" ::"s"(a.n_ee));   // (in the first kernarg batch: read later, in mode 0)
  const int D = a.D, nt = D / 32, nblk = nt * nt, t = threadIdx.x, b = blockIdx.x;
  const int mode = a.mode, it = a.it;
  FrSched* sc = a.sc;
  // Everything before the product's first wait is issued at once: the skip flag,
  // the product's first stage, then the epilogue's inputs -- the scalars' partials
  // of the previous launches and this block's own entries of the CG vectors (only
  // this block writes them; the product reads the whole operand, which no block of
  // this launch writes).  All straight-line loads at clamped indices (entry 1 of a
  // half block re-reads entry 0; sources a mode does not use read another vector),
  // so no wait precedes them.  Iterations past convergence then return (every wave
  // reads the flag itself; a flag holding this launch's own tag was set by a peer
  // block and is ignored).
  // (a per-lane load: the compiler moves a uniform one to a scalar register, and
  // waits for it, right where it is loaded)
  int lane0;
  asm volatile("v_mov_b32 %0, 0" : "=v"(lane0));
  const int fv = __hip_atomic_load(&sc->pcg_done + lane0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const Geo g = geo_xcd(b, nt);
  const int nown = n_own(g);
  long long idx[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = t + NTH * (k < nown ? k : 0), r = e >> 5, c = e & 31;
    idx[k] = (long long)(g.r0 + r) * D + g.c0 + c;
  }
  const double* pa1 = mode == 0 ? a.ee_part : a.gam + (it & 1) * nblk;
  const double* pa2 = mode == 1 ? a.gam + ((it > 0 ? it - 1 : 0) & 1) * nblk : a.pi;
  const int n1 = mode == 0 ? (b == 0 ? a.n_ee : 0) : nblk;
  const int n2 = (mode == 1 && it >= 1) || mode == 2 ? nblk : 0;
  const int n3 = mode == 1 && it >= 1 ? nblk : 0;
  PartLoad l1, l2, l3;
  // own entries o[j]: mode 0 R; mode 1 U, P, Q (it >= 1); mode 2 P, Q, R, U, X (it >= 1)
  const double* src[5] = {mode == 0 ? a.R : (mode == 1 ? a.U : a.P), mode == 1 ? a.P : a.Q,
                          mode == 1 ? a.Q : a.R, a.U, a.X};
  double o[5][2];
#ifdef VB_SS_PROF
  unsigned long long pst[6];
#endif
  const bool go = product<KT>(a.Mat, a.V, D, g, lds, [&]() {
    // (after the first stage's loads were issued)
    l1.load(pa1, n1);
    l2.load(pa2, n2);
    l3.load(a.rho, n3);
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int k = 0; k < 2; ++k) o[j][k] = src[j][idx[k]];
#ifdef VB_SS_PROF
    pst[2] = __builtin_amdgcn_s_memrealtime();
#endif
    const int f = mode != 0 ? __builtin_amdgcn_readfirstlane(fv) : 0;
    return !(f != 0 && !(mode == 1 && f == it + 1));
  }
#ifdef VB_SS_PROF
  , pst
#endif
  );
  if (!go) return;
#ifdef VB_SS_PROF
  pst[3] = __builtin_amdgcn_s_memrealtime();
#endif
  // the scalars (gamma_i, gamma_{i-1} or pi_i, ||R_i||^2), summed by each wave
  const double sc3[3] = {l1.total(pa1, n1), l2.total(pa2, n2), l3.total(a.rho, n3)};
#ifdef VB_SS_PROF
  pst[4] = __builtin_amdgcn_s_memrealtime();
#endif
  if (mode == 1 && it >= 1) {
    // A_i tests R_i (M_{i-1}'s partials) after its product: with the learnt
    // iteration count the test usually fails, so it stays off the launch's
    // critical path; a converged launch writes nothing.  Every block sums the
    // same partials in the same order and decides alike.
    if (sc3[2] <= a.tol2 * sc->ee) {
      if (t == 0) {
        sc->pcg_iter = it - 1;
        __hip_atomic_store(&sc->pcg_done, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  double* vt = lds + RED;               // the block's result entries (stride VS)
  double* xt = vt + 32 * VS;            // mode 2: X's new entries (mirror staging)
  const double wgt = own_weight(g);
  double acc[2] = {0.0, 0.0};
  if (mode == 0) {
    if (b == 0 && t == 0) sc->ee = sc3[0] * sc->ee_scale;
    for (int k = 0; k < nown; ++k) {
      const int e = t + NTH * k, r = e >> 5, c = e & 31;
      const double u = 0.25 * vt[r * VS + c];
      vt[r * VS + c] = u;
      a.U[idx[k]] = u;
      acc[0] = fma(o[0][k], u, acc[0]);
    }
    double red1[1] = {wgt * acc[0]};
    block_sum8v(red1, scr);
    if (t == 0) a.gam[b] = red1[0];
  } else if (mode == 1) {
    const double beta = it >= 1 ? sc3[0] / sc3[1] : 0.0;
    for (int k = 0; k < nown; ++k) {
      const int e = t + NTH * k, r = e >> 5, c = e & 31;
      const double w = vt[r * VS + c];
      const double p = it >= 1 ? fma(beta, o[1][k], o[0][k]) : o[0][k];
      const double q = it >= 1 ? fma(beta, o[2][k], w) : w;
      vt[r * VS + c] = q;
      a.P[idx[k]] = p;
      a.Q[idx[k]] = q;
      acc[0] = fma(p, q, acc[0]);
    }
    double red1[1] = {wgt * acc[0]};
    block_sum8v(red1, scr);   // (its barriers also complete vt)
    if (t == 0) a.pi[b] = red1[0];
  } else {
    const double alpha = sc3[0] / sc3[1];
    for (int k = 0; k < nown; ++k) {
      const int e = t + NTH * k, r = e >> 5, c = e & 31;
      const double v = 0.25 * vt[r * VS + c];
      const double x = it >= 1 ? fma(alpha, o[0][k], o[4][k]) : alpha * o[0][k];
      const double rn = fma(-alpha, o[1][k], o[2][k]), un = fma(-alpha, v, o[3][k]);
      vt[r * VS + c] = un;
      xt[r * VS + c] = x;
      a.X[idx[k]] = x;
      a.R[idx[k]] = rn;
      a.U[idx[k]] = un;
      acc[0] = fma(rn, un, acc[0]);
      acc[1] = fma(rn, rn, acc[1]);
    }
    acc[0] *= wgt;
    acc[1] *= wgt;
    block_sum8v(acc, scr);
    if (t == 0) {
      a.gam[((it + 1) & 1) * nblk + b] = acc[0];
      a.rho[b] = acc[1];
    }
  }
  // mirror entries of the operands of later products (U, Q) and of X: thread t
  // -> column c, row r of the transposed half (block_sum8's barriers ordered the
  // staged entries above)
  if (!g.diag) {
    const int c = t >> 4, r = t & 15;
    const long long m = (long long)(g.c0 + c) * D + g.r0 + r;
    const double v = vt[r * VS + c];
    if (mode == 0 || mode == 2) a.U[m] = v;
    if (mode == 1) a.Q[m] = v;
    if (mode == 2) a.X[m] = xt[r * VS + c];
  }
#ifdef VB_SS_PROF
  // one line per block of every launch of the VB_SS_PROF-th PCG call (entry
  // stamp, first batch issued, first stage landed, main loop done, product done,
  // scalars summed, end; CU id from HW_ID)
  pst[5] = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    if (a.pcg_call == VB_SS_PROF)
      printf("SSPROF %d %d %d %u %llu %llu %llu %llu %llu %llu %llu\n", mode, it, b,
             __builtin_amdgcn_s_getreg(63508), p_entry, pst[2], pst[0], pst[1], pst[3], pst[4],
             pst[5]);
  }
#endif
}

}  // namespace

// ---- workspace ---------------------------------------------------------------
struct FrWork {
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
      if (bytes <= cap) return hipSuccess;
      if (p) (void)hipFree(p);
      p = nullptr;
      cap = 0;
      hipError_t e = hipMalloc(&p, bytes);
      if (e == hipSuccess) cap = bytes;
      return e;
    }
    double* d() const { return static_cast<double*>(p); }
    ~Buf() {
      if (p) (void)hipFree(p);
    }
  };
  rocblas_handle blas = nullptr;
  int D = 0;
  // D x D
  Buf L, E, T, GS, H, Sig, Yb[2], Zb[2], Eh, Xs, R, P, C1, C2;
  // D
  Buf w, offd, scal, pv[4];
  Buf info, sched, fro_part, tpart[2], pq_part, rz_part, rr_part, ee_part;
  // stream-K scratch of the Newton-Schulz Y|Z launches (GemmOp::sk_part / sk_flag):
  // a partial tile and a flag per upper-triangle tile of the pair; sk_epoch tags
  // each launch (flags start at 0)
  Buf sk_part, sk_flag;
  int sk_epoch = 0;
  FrSched* host_sched = nullptr;  // pinned copy of the schedule / status block
  const double* Yf = nullptr;     // final Newton-Schulz iterates (A^(1/2), A^(-1/2))
  const double* Zf = nullptr;
  bool have_z = false;            // Zf holds a previous root (power-iteration start)
  int pv_cur = 0;                 // power-iteration vectors: pv[pv_cur] (Sigma), pv[2 + pv_cur] (Z)
  bool warm = false;              // pv hold the previous root's vectors
  bool zv_init = false;           // pv[2..3] hold a Z power vector
  bool last_warm = false;         // the last root was a warm one (iteration hints apply)
  const void* owner = nullptr;    // the run whose root the warm state above holds
  int ns_kmax = 12, pcg_kmax = 14;  // iterations launched (device skips past convergence)
  int last_kmax = 12;             // Newton-Schulz iterations the last root launched
  int retry_kmax = 0;             // Newton-Schulz floor after a call / advance ran again
  int retry_pcg = 0;              // PCG floor after a call / advance ran again
  const void* retry_owner = nullptr;  // the run the floors belong to
  int kpcg_max_seen = 0;          // most PCG iterations launched since the last fr_info
  int pcg_last = 0;               // the last PCG call: index of its last launched iteration
  int pcg_calls = 0;              // symmetric-sum PCG calls so far (VB_SS_PROF)
  double pcg_tol2 = 1e-18;        // and its convergence bar (||R||^2 / ||E||^2)
  bool eig_pending = false;       // a dsyevd ran since the last fr_info
  bool sqrt_pending = false;      // a Newton-Schulz / PCG status to read at fr_info
  bool last_hz = false;           // the last root's schedule had a Z power vector (uZ valid)
  int c_slot = 0;                 // FrSched::cbuf slot the last schedule wrote
  // fused steps (fr_value_grad with an adagrad update and Philox draws): the last
  // step's final kernel prepared the next one -- L of the updated parameters, the
  // draws (Z, s, zz) of rng step prep_step on (prep_k0, prep_k1, prep_stream) and
  // the power step pz = Z u -- for prep_owner; any other use of the workspace
  // clears prep_owner
  const void* prep_owner = nullptr;
  long long prep_step = -1;
  uint32_t prep_k0 = 0, prep_k1 = 0, prep_stream = 0;
  Buf uS, uZ, pS, pz, ypart, lp_part;
  // fr_warm_save / fr_warm_restore: the warm state an advance starts from
  // (device: uS, uZ, pv[0..3], the previous root Z, the schedule block; host:
  // the flags below), so an advance that runs again starts where it started
  Buf wsnap;
  struct WarmHost {
    bool warm, have_z, zv_init, last_hz, valid;
    int pv_cur, zf_slot, c_slot;
    const void* owner;
  } wsnap_h{};
  // N x D / N
  Buf Z, X, G, s, logp, zz, r, rk;
  // pinned host staging for host-callback targets
  double *hx = nullptr, *hlp = nullptr, *hg = nullptr;
  size_t hcap = 0;
  ~FrWork() {
    if (blas) rocblas_destroy_handle(blas);
    if (host_sched) (void)hipHostFree(host_sched);
    for (double* p : {hx, hlp, hg})
      if (p) (void)hipHostFree(p);
  }
};

FrWork* fr_work_create() { return new (std::nothrow) FrWork(); }
void fr_work_destroy(FrWork* w) { delete w; }

namespace {

// VIABEL_AMD_FR_PCG_SS=0: the PCG runs its products and vector updates as separate
// launches (pcg_xr / pcg_p) even where the symmetric-sum loop applies (A/B switch)
bool pcg_ss_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_FR_PCG_SS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// VIABEL_AMD_FR_SCHED_FUSE=0: the schedule kernel runs on its own (A/B switch)
bool sched_fused() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_FR_SCHED_FUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

#define FR_HIP(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return vb_set_error(e_ == hipErrorOutOfMemory ? -3 : -2, "%s failed: %s (%s:%d)", #expr, \
                          hipGetErrorString(e_), __FILE__, __LINE__);                      \
  } while (0)

int reserve_d(FrWork* W, int D, hipStream_t st) {
  if (!W->blas) {
    if (rocblas_create_handle(&W->blas) != rocblas_status_success)
      return vb_set_error(-2, "rocblas_create_handle failed");
  }
  if (rocblas_set_stream(W->blas, st) != rocblas_status_success)
    return vb_set_error(-2, "rocblas_set_stream failed");
  if (W->D >= D) return 0;
  const size_t dd = sizeof(double) * (size_t)D * D;
  for (FrWork::Buf* b : {&W->L, &W->E, &W->T, &W->GS, &W->H, &W->Sig, &W->Yb[0], &W->Yb[1],
                         &W->Zb[0], &W->Zb[1], &W->Eh, &W->Xs, &W->R, &W->P, &W->C1, &W->C2})
    FR_HIP(b->reserve(dd));
  for (FrWork::Buf* b : {&W->w, &W->offd, &W->pv[0], &W->pv[1], &W->pv[2], &W->pv[3], &W->uS,
                         &W->uZ, &W->pS, &W->pz})
    FR_HIP(b->reserve(sizeof(double) * D));
  FR_HIP(W->ypart.reserve(sizeof(double) * 4 * ((D + 31) / 32) * ((D + 31) / 32)));
  FR_HIP(W->scal.reserve(sizeof(double) * 8));
  FR_HIP(W->info.reserve(sizeof(int) * 4));
  const size_t nblk = (size_t)((D + 31) / 32) * ((D + 31) / 32);
  for (FrWork::Buf* b : {&W->fro_part, &W->tpart[0], &W->tpart[1], &W->pq_part, &W->rz_part})
    FR_HIP(b->reserve(sizeof(double) * 4 * nblk));
  for (FrWork::Buf* b : {&W->rr_part, &W->ee_part}) FR_HIP(b->reserve(sizeof(double) * nblk));
  {
    const size_t nt = (size_t)((D + 31) / 32), npair = nt * (nt + 1);   // tiles of the Y|Z pair
    FR_HIP(W->sk_part.reserve(sizeof(double) * 1024 * npair));
    FR_HIP(W->sk_flag.reserve(sizeof(int) * npair));
    FR_HIP(hipMemsetAsync(W->sk_flag.p, 0, sizeof(int) * npair, st));
    W->sk_epoch = 0;
  }
  if (!W->sched.p) {
    FR_HIP(W->sched.reserve(sizeof(FrSched)));
    FR_HIP(hipMemsetAsync(W->sched.p, 0, sizeof(FrSched), st));
  }
  if (!W->host_sched) FR_HIP(hipHostMalloc(&W->host_sched, sizeof(FrSched)));
  W->warm = false;
  W->have_z = false;
  W->zv_init = false;
  W->D = D;
  return 0;
}

int reserve_n(FrWork* W, int D, long long n) {
  const size_t nd = sizeof(double) * (size_t)n * D, n1 = sizeof(double) * (size_t)std::max(n, 1LL);
  FR_HIP(W->Z.reserve(nd));
  FR_HIP(W->X.reserve(nd));
  FR_HIP(W->G.reserve(nd));
  for (FrWork::Buf* b : {&W->s, &W->logp, &W->zz, &W->r, &W->rk}) FR_HIP(b->reserve(n1));
  FR_HIP(W->lp_part.reserve(n1 * 2 * ((D + 31) / 32)));
  return 0;
}

}  // namespace

int host_target_eval(FrWork* W, const HostTarget& t, int D, long long n, const double* x,
                     double* logp, double* grad, hipStream_t st) {
  if (!t.fn) return vb_set_error(-1, "callback target without a callback");
  const size_t nd = (size_t)n * D;
  if (nd > W->hcap || (size_t)n > W->hcap) {
    for (double** p : {&W->hx, &W->hlp, &W->hg}) {
      if (*p) (void)hipHostFree(*p);
      *p = nullptr;
    }
    W->hcap = 0;
    const size_t cap = std::max(nd, (size_t)n);
    for (double** p : {&W->hx, &W->hlp, &W->hg}) FR_HIP(hipHostMalloc(p, sizeof(double) * cap));
    W->hcap = cap;
  }
  FR_HIP(hipMemcpyAsync(W->hx, x, sizeof(double) * nd, hipMemcpyDefault, st));
  FR_HIP(hipStreamSynchronize(st));
  const int rc = t.fn(t.user, W->hx, (int64_t)n, (int64_t)D, W->hlp, W->hg);
  if (rc != 0) return vb_set_error(-2, "target callback returned %d", rc);
  FR_HIP(hipMemcpyAsync(logp, W->hlp, sizeof(double) * n, hipMemcpyDefault, st));
  if (grad) FR_HIP(hipMemcpyAsync(grad, W->hg, sizeof(double) * nd, hipMemcpyDefault, st));
  // the staging buffers are reused by the next call, which synchronises first
  return 0;
}

namespace {
int eval_target(FrWork* W, int tgt, const HostTarget& host, int D, long long n, const double* x,
                double* logp, double* grad, hipStream_t st) {
  if (tgt == kTargetCallback) return host_target_eval(W, host, D, n, x, logp, grad, st);
  FR_HIP(launch_target_logdensity(tgt, D, n, x, logp, grad, st));
  return 0;
}
}  // namespace

// L, eigh(L L^T) -> (w ascending, Vt rows = eigenvectors), half log det from the
// eigenvalues (multivariate_t_logpdf's log_pdet, _distributions.py:27-32)
int fr_prepare(FrWork* W, int D, const double* lam, hipStream_t st) {
  W->prep_owner = nullptr;
  if (int rc = reserve_d(W, D, st)) return rc;
  hipLaunchKernelGGL(fr_unpack_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, lam,
                     W->L.d());
  FR_HIP(gemm(mm(D, D, D, W->L.d(), false, W->L.d(), true, W->E.d()), st));
  // rocSOLVER is column-major: the symmetric input reads the same either way;
  // eigenvector k comes back as column k, i.e. row k of our row-major view.
  rocblas_status rs = rocsolver_dsyevd(W->blas, rocblas_evect_original, rocblas_fill_upper, D,
                                       W->E.d(), D, W->w.d(), W->offd.d(),
                                       static_cast<rocblas_int*>(W->info.p));
  if (rs != rocblas_status_success) return vb_set_error(-2, "rocsolver_dsyevd failed (%d)", (int)rs);
  W->eig_pending = true;
  hipLaunchKernelGGL(fr_logdet_kernel, dim3(1), dim3(1024), 0, st, D, W->w.d(), W->scal.d());
  FR_HIP(hipGetLastError());
  return 0;
}

// S = sqrtm(Sigma) without an eigendecomposition and without a host round trip:
// scaled coupled Newton-Schulz (FrSched above).  Launches: Sigma = L L^T (its
// epilogue gives ||Sigma||_F^2), n_pow power steps on Sigma and on the previous
// root's Z, the schedule kernel, iteration 0 (one GEMM: Y_1, Z_1 are polynomials
// in Sigma), then for k = 1 .. ns_kmax: T_k (its epilogue gives ||I - Z_k Y_k||_F
// partials) and the grouped Y_{k+1}, Z_{k+1} product, whose blocks first test
// convergence (||I - Z_k Y_k||_F <= 1e-10 sqrt(D), or a rounding-floor stall
// below 1e-8 sqrt(D)) and then copy Y_k, Z_k through instead; later T GEMMs
// return at once.  Non-convergence within ns_kmax sets FrSched::status (read by
// fr_info).  `warm`: Sigma is close to the previous call's (an optimisation
// run), so 3 warm-started power steps suffice and l_0 comes from the previous
// root; otherwise 8 power steps from ones and l_0 = 0.05.
// Also: L, Sigma = L L^T, scal[0] = 0.5 log det Sigma = sum log L_ii.
// `ready` (a fused step prepared by the previous one, see FrWork::prep_owner): L
// is current and the power steps (pS = Sigma_prev uS, pz = Z_prev uZ) came from
// the previous step's last kernel; the Sigma GEMM's epilogue gives the Rayleigh
// quotient partials of pS, so no unpack and no power launches.
int fr_sqrt(FrWork* W, int D, const double* lam, hipStream_t st, bool warm, const void* owner,
            bool ready) {
  if (!ready) W->prep_owner = nullptr;   // L, Sigma, the root and uS change below
  if (int rc = reserve_d(W, D, st)) return rc;
  const long long dd = (long long)D * D;
  // every product here is symmetric (polynomials in Sigma): upper-triangle tiles
  // only (GemmOp::sym), with gemm_parts(D, true) partial sums
  const int nparts = gemm_parts(D, true);
  FrSched* sc = static_cast<FrSched*>(W->sched.p);
  if (!ready)
    hipLaunchKernelGGL(fr_unpack_kernel, dim3(blocks(dd)), dim3(256), 0, st, D, lam, W->L.d());
  {
    GemmOp g = mm(D, D, D, W->L.d(), false, W->L.d(), true, W->Sig.d());
    g.sym = 1;
    g.sq_part = W->fro_part.d();
    if (ready) {   // Rayleigh quotient partials of the previous step's Sigma uS
      g.qf_x = W->pS.d();
      g.qf_part = W->ypart.d();
    }
    FR_HIP(gemm(g, st));
  }
  // power steps: Sigma x and Z_prev u (the previous root's vectors as start).
  // Warm state (previous root, power vectors, learnt iteration counts) belongs
  // to the run that made it: any other caller's root (another run, a cold
  // log-weight or single-call root) invalidates it
  warm = warm && W->warm && owner != nullptr && W->owner == owner;
  if (W->owner != owner && W->retry_owner != owner) W->retry_kmax = W->retry_pcg = 0;
  W->owner = owner;
  // a cold root starts a new problem: forget the iteration counts learnt on the
  // previous one (fr_info learns them again from this run's warm steps)
  if (!warm) {
    // (VIABEL_AMD_FR_NS_START: test hook -- the count warm roots start from before
    // fr_info has learnt one, e.g. too few to exercise the advance retry)
    const char* e = std::getenv("VIABEL_AMD_FR_NS_START");
    W->ns_kmax = e ? std::max(1, std::atoi(e)) : 12;
    W->pcg_kmax = 14;
    // and its first warm step starts the Z power vector afresh (not from a vector
    // another problem left in the workspace): a run's steps then depend only on
    // the run, whatever used the workspace before it
    W->zv_init = false;
  }
  const bool hz = warm && W->have_z && W->Zf;
  const int n_pow = ready ? 0 : warm ? 3 : 8;
  const unsigned nb = (unsigned)((D + 7) / 8);
  for (int p = 0; p < n_pow; ++p) {
    const int a = W->pv_cur, b = 1 - a;
    const bool xfirst = p == 0 && !warm, ufirst = p == 0 && !W->zv_init;
    // a warm start begins from the last sched's unit vectors (fused steps in
    // between updated them, not pv)
    const double* xin = xfirst ? nullptr : (p == 0 ? W->uS.d() : W->pv[a].d());
    const double* uin = ufirst ? nullptr : (p == 0 && W->last_hz ? W->uZ.d() : W->pv[2 + a].d());
    hipLaunchKernelGGL(fr_power2_kernel, dim3(nb, hz ? 2 : 1), dim3(256), 0, st, D, W->Sig.d(),
                       xin, W->pv[b].d(), W->Zf, uin, W->pv[2 + b].d());
    W->pv_cur = b;
  }
  if (hz) W->zv_init = true;
  // warm roots launch exactly the learnt count (fr_info; a step that needs more
  // sets the sticky status and, inside a run's advance, makes the advance run
  // again with a larger count -- vb_run_advance keeps a snapshot), others at
  // least 12 (l_0 = 0.05 needs ~9 at rounding level)
  const int kmax =
      std::min(warm ? std::max({W->ns_kmax, W->retry_kmax, 3})
                    : std::max({W->ns_kmax + 1, 12, W->retry_kmax}),
               kFrNSMax);
  W->last_warm = warm;
  W->last_kmax = kmax;
  W->c_slot ^= 1;
  SchedArgs sh{};
  sh.D = D;
  sh.kmax = kmax;
  sh.n_part = nparts;
  sh.has_z = ready || hz ? 1 : 0;
  sh.slot = W->c_slot;
  sh.l_default = 0.05;
  sh.fro_part = W->fro_part.d();
  sh.qf_part = ready ? W->ypart.d() : nullptr;
  sh.y = ready ? W->pS.d() : W->pv[W->pv_cur].d();
  sh.v = ready ? W->pz.d() : W->pv[2 + W->pv_cur].d();
  sh.lam = lam;
  sh.sc = sc;
  sh.scal = W->scal.d();
  sh.uS = W->uS.d();
  sh.uZ = W->uZ.d();
  W->last_hz = ready || hz;
  // iteration 0: Y_1 -> Yb[1], Z_1 -> Zb[1]; the schedule is computed inside it
  // (SchedHook) when the shapes allow, else by its own kernel first
  GemmOp g0 = mm(D, D, D, W->Sig.d(), false, W->Sig.d(), false, W->Yb[1].d());
  g0.sym = 1;
  g0.ns0_z = W->Zb[1].d();
  if (sched_fused() && D <= kSchedHookMaxD && nparts <= kSchedP * 512 && gemm_detail::glds_ok_shape(g0)) {
    g0.ns0 = sc->ns0;   // (marks the iteration-0 epilogue; the hook's block-local copy is used)
    FR_HIP(gemm_hook<SchedHook>(g0, sh, st));
  } else {
    hipLaunchKernelGGL(fr_sched_kernel, dim3(1), dim3(1024), 0, st, D, kmax, sh.fro_part, nparts,
                       sh.y, sh.v, sh.has_z, sh.l_default, sc, lam, sh.scal, sh.qf_part, sh.uS,
                       sh.uZ, sh.slot);
    g0.ns0 = sc->ns0;
    FR_HIP(gemm(g0, st));
  }
  for (int k = 1; k <= kmax; ++k) {
    const double *Yk = W->Yb[k & 1].d(), *Zk = W->Zb[k & 1].d();
    double* tp = W->tpart[k & 1].d();
    GemmOp t = mm(D, D, D, Zk, false, Yk, false, W->T.d());
    t.sym = 1;
    t.alpha_dev = &sc->nalpha2[k];
    t.diag = 3.0;
    t.sq_part = tp;
    t.sq_shift_dev = &sc->shift[k];
    t.skip_flag = &sc->ns_conv;
    t.skip_tag = 2 * k + 1;
    t.skip_flag2 = &sc->ns_fin;
    FR_HIP(gemm(t, st));
    GemmOp yz[2] = {mm(D, D, D, Yk, false, W->T.d(), false, W->Yb[(k + 1) & 1].d()),
                    mm(D, D, D, W->T.d(), false, Zk, false, W->Zb[(k + 1) & 1].d())};
    for (int o = 0; o < 2; ++o) {
      GemmOp& g = yz[o];
      g.sym = 1;
      g.alpha_dev = &sc->halpha[k];
      g.skip_flag = &sc->ns_conv;
      g.skip_tag = 2 * k + 2;
      // the root ends in buffer (kmax + 1) & 1: the first skipped launch copies
      // it there when it sits in the other one
      g.copy_src = ((k & 1) != ((kmax + 1) & 1)) ? (o == 0 ? Yk : Zk) : nullptr;
      g.copy_if_iter = k;
      g.conv_part = tp;
      g.conv_n = nparts;
      g.conv_scale_dev = &sc->inv_a4[k];
      g.conv_tol2 = 1e-20 * D;
      // ||I - Z_k Y_k||_F <= tau: the residual after this update is at most
      // 0.75 ||E||_F ||E||_2 <= 0.75 tau^2 (e' = (3 e^2 + e^3) / 4 per
      // eigenvalue), so with tau^2 = 0.67e-10 sqrt(D) (half the largest tau that
      // keeps 0.75 tau^2 below the 1e-10 sqrt(D) bar) this update is the last
      // one: the detection-only T_{k+1} product and the Y|Z launch after it are
      // saved, and the root is the same iterate
      g.fin_flag = &sc->ns_fin;
      g.conv_fin_tol2 = 0.67e-10 * std::sqrt((double)D);
      if (k >= 2) {
        g.conv_prev_part = W->tpart[(k - 1) & 1].d();
        g.conv_prev_scale_dev = &sc->inv_a4[k - 1];
        g.conv_stall_tol2 = 1e-16 * D;
      }
      g.conv_iter_out = &sc->ns_iter;
      g.conv_iter = k;
    }
    // stream-K scratch (gemm_group takes it where the tile count suits, D = 512)
    const int epoch = ++W->sk_epoch > 0 ? W->sk_epoch : (W->sk_epoch = 1);
    for (GemmOp& g : yz) {
      g.sk_part = W->sk_part.d();
      g.sk_flag = static_cast<int*>(W->sk_flag.p);
      g.sk_epoch = epoch;
    }
    FR_HIP(gemm_group(yz, 2, st));
  }
  W->Yf = W->Yb[(kmax + 1) & 1].d();
  W->Zf = W->Zb[(kmax + 1) & 1].d();
  W->have_z = true;
  W->warm = true;
  W->sqrt_pending = true;
  FR_HIP(hipGetLastError());
  return 0;
}

// Preconditioned conjugate gradients for autograd's sqrtm VJP (see pcg_* above):
// X = the symmetric solution of S X + X S = G_S + G_S^T, into W->Xs.
// (gmu non-null: the init launch also reduces the mean gradient gmu = r^T Gm,
// N x D, in an extra row of blocks.)
int fr_pcg(FrWork* W, int D, hipStream_t st, int N = 0, const double* rw = nullptr,
           const double* Gm = nullptr, double* gmu = nullptr) {
  FrSched* sc = static_cast<FrSched*>(W->sched.p);
  const int nt = (D + kTile - 1) / kTile, nblk = nt * nt;
  const dim3 tg(nt, nt);
  const int n_cs = gmu ? (D + 63) / 64 : 0;
  hipLaunchKernelGGL(pcg_init_kernel, dim3(nt, nt + (n_cs ? 1 : 0)), dim3(256), 0, st, D,
                     W->GS.d(), sc, W->Eh.d(), W->R.d(), W->Xs.d(), W->ee_part.d(), n_cs, N, rw,
                     Gm, gmu);
  // warm roots launch the learnt count (fr_info), others at least 16; a rerun
  // after a residual above the status bar launches at least its floor
  const int kpcg = std::min(kFrPcgMax, std::max(W->last_warm ? std::max(W->pcg_kmax, 3)
                                                             : std::max(W->pcg_kmax, 16),
                                                W->retry_pcg));
  W->kpcg_max_seen = std::max(W->kpcg_max_seen, kpcg);
  // converged when ||R|| <= tol ||E||: X then carries at most the preconditioned
  // condition number (< 1.2 at config 4) x tol of relative error.  tol = 1e-9 for
  // cold roots (single value-and-gradient calls), 1e-8 for the warm steps of an
  // optimisation run (one CG iteration fewer at config 4; still three orders
  // inside the 1e-5 parity bar of north_star, and far below the step's Monte
  // Carlo noise); the sticky status flags residuals above 1e-7 (a learnt count
  // one short)
  const double tol2 = W->last_warm ? 1e-16 : 1e-18;
  W->pcg_last = kpcg - 1;
  W->pcg_tol2 = tol2;
  if (symsum::usable(D, W->Zf, W->R.d()) && symsum::usable(D, W->Yf, W->Xs.d()) &&
      pcg_ss_enabled()) {
    // symmetric-sum products with the updates in their epilogues (fr_pcg_ss_kernel)
    SsPcgArgs a{};
    a.D = D;
    a.R = W->R.d();
    a.U = W->C2.d();
    a.P = W->P.d();
    a.Q = W->C1.d();
    a.X = W->Xs.d();
    a.ee_part = W->ee_part.d();
    a.n_ee = nblk;
    a.gam = W->rz_part.d();
    a.pi = W->pq_part.d();
    a.rho = W->rr_part.d();
    a.sc = sc;
    a.tol2 = tol2;
    a.pcg_call = W->pcg_calls++;
    const dim3 grid((unsigned)((D / 32) * (D / 32)));
    auto launch = [&]() {
      gemm_flop_tally() += 2.0 * D * (double)D * D;   // nt^2 blocks x 16 x 32 x 2D x 2
      if (symsum::kt_for(D) == 128)
        hipLaunchKernelGGL(fr_pcg_ss_kernel<128>, grid, dim3(symsum::NTH), symsum::Cfg<128>::LDS_BYTES,
                           st, a);
      else
        hipLaunchKernelGGL(fr_pcg_ss_kernel<64>, grid, dim3(symsum::NTH), symsum::Cfg<64>::LDS_BYTES,
                           st, a);
    };
    a.mode = 0;
    a.it = 0;
    a.Mat = W->Zf;
    a.V = a.R;
    launch();
    for (int it = 0; it < kpcg; ++it) {
      a.it = it;
      a.mode = 1;
      a.Mat = W->Yf;
      a.V = a.U;
      launch();
      a.mode = 2;
      a.Mat = W->Zf;
      a.V = a.Q;
      launch();
    }
    FR_HIP(hipGetLastError());
    return 0;
  }
  // P_0 = M^-1(R_0) from C2 = Z R_0, <R_0, Z R_0> in the epilogue
  auto zr = [&](int it) {
    GemmOp g = mm(D, D, D, W->Zf, false, W->R.d(), false, W->C2.d());
    g.dot_with = W->R.d();
    g.dot_part = W->rz_part.d();
    g.skip_flag = &sc->pcg_done;
    // (the tolerance: see above)
    if (it >= 0) {
      g.conv_part = W->rr_part.d();
      g.conv_n = nblk;
      g.conv_ref_dev = &sc->ee;
      g.conv_tol2 = tol2;
      g.conv_iter_out = &sc->pcg_iter;
      g.conv_iter = it;
      g.skip_tag = it + 1;
    }
    return g;
  };
  FR_HIP(gemm(zr(-1), st));
  hipLaunchKernelGGL(pcg_p_kernel, tg, dim3(256), 0, st, D, -1, W->C2.d(), W->rz_part.d(),
                     4 * nblk, W->ee_part.d(), nblk, sc, W->P.d());
  for (int it = 0; it < kpcg; ++it) {
    GemmOp g = mm(D, D, D, W->Yf, false, W->P.d(), false, W->C1.d());
    g.dot_with = W->P.d();
    g.dot_part = W->pq_part.d();
    g.skip_flag = &sc->pcg_done;
    FR_HIP(gemm(g, st));
    hipLaunchKernelGGL(pcg_xr_kernel, tg, dim3(256), 0, st, D, it, W->C1.d(), W->P.d(),
                       W->pq_part.d(), 4 * nblk, sc, W->Xs.d(), W->R.d(), W->rr_part.d());
    FR_HIP(gemm(zr(it), st));
    hipLaunchKernelGGL(pcg_p_kernel, tg, dim3(256), 0, st, D, it, W->C2.d(), W->rz_part.d(),
                       4 * nblk, W->ee_part.d(), nblk, sc, W->P.d());
  }
  FR_HIP(hipGetLastError());
  return 0;
}

// s (n) and z (n x D) into the workspace; host_eps = [s (n), z (n x D)] on the device
int fr_draw(FrWork* W, int D, long long n, double df, const double* host_eps, uint32_t k0,
            uint32_t k1, uint32_t stream, uint32_t step, const double** s_out,
            const double** z_out, hipStream_t st) {
  W->prep_owner = nullptr;
  if (host_eps) {
    *s_out = host_eps;
    *z_out = host_eps + n;
    return 0;
  }
  if (int rc = reserve_n(W, D, n)) return rc;
  Rng rng{k0, k1, stream};
  const long long tot = n * ((D + 1) / 2 + 1);
  hipLaunchKernelGGL(fr_noise_kernel, dim3(blocks(tot)), dim3(256), 0, st, D, n, rng, step, df,
                     W->Z.d(), W->s.d());
  FR_HIP(hipGetLastError());
  *s_out = W->s.d();
  *z_out = W->Z.d();
  return 0;
}

// x = mu + (z S) / s, S = sqrt(c) Y_final  (after fr_sqrt)
int fr_transform(FrWork* W, int D, long long n, const double* mu, const double* s,
                 const double* z, double* x, hipStream_t st) {
  GemmOp g = mm((int)n, D, D, z, false, W->Yf, false, x);
  g.alpha_dev = &static_cast<FrSched*>(W->sched.p)->sqrt_c;
  g.row_div = s;
  g.col_bias = mu;
  FR_HIP(gemm(g, st));
  return 0;
}

// log p and gradient of a target at x (n x D)
int fr_target(FrWork* W, int tgt, int D, long long n, const double* tparams, double tconst,
              const double* x, double* logp, double* G, hipStream_t st) {
  if (tgt == kTargetCorrGauss) {
    double* g = G;
    if (!g) {
      if (int rc = reserve_n(W, D, n)) return rc;
      g = W->G.d();
    }
    FR_HIP(gemm(mm((int)n, D, D, x, false, tparams, false, g, -1.0), st));
    hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(n, 4)), dim3(256), 0, st, D, n, nullptr, x, g,
                       tconst, 1, nullptr, logp);
    FR_HIP(hipGetLastError());
    return 0;
  }
  FR_HIP(launch_target_logdensity(tgt, D, n, x, logp, G, st));
  return 0;
}

// One KLVI / CHIVI value + gradient (vb.py:236-266) at lam, gradient into grad[P]
// and the value into *value (device pointers).
int fr_value_grad(FrWork* W, const FrSpec& f, const double* lam, const double* host_eps,
                  uint32_t k0, uint32_t k1, uint32_t stream, uint32_t step, double* value,
                  double* grad, hipStream_t st, bool warm, const void* owner,
                  const MfUpdate* up, const FrNext* next) {
  const int D = f.D, N = f.N;
  // fused step: adagrad in the last kernel, Philox draws reduced with zz by their
  // own kernel, logp (corr_gauss) from the target GEMM's row partials, the mean
  // gradient in pcg_init's extra blocks; `ready`: the previous fused step of this
  // run already prepared L, the draws and the Z power step (FrWork::prep_owner)
  const bool fused = up != nullptr && host_eps == nullptr;
  const bool ready = fused && warm && owner != nullptr && W->prep_owner == owner &&
                     W->prep_step == (long long)step && W->prep_k0 == k0 && W->prep_k1 == k1 &&
                     W->prep_stream == stream;
  W->prep_owner = nullptr;
  if (int rc = fr_sqrt(W, D, lam, st, warm, owner, ready)) return rc;
  if (int rc = reserve_n(W, D, N)) return rc;
  const double *s, *z;
  if (ready) {
    s = W->s.d();
    z = W->Z.d();
  } else if (fused) {
    hipLaunchKernelGGL(fr_noise_rows_kernel, dim3(N), dim3(256), 0, st, D, Rng{k0, k1, stream},
                       step, f.df, W->Z.d(), W->s.d(), W->zz.d());
    s = W->s.d();
    z = W->Z.d();
  } else if (int rc = fr_draw(W, D, N, f.df, host_eps, k0, k1, stream, step, &s, &z, st)) {
    return rc;
  }
  if (int rc = fr_transform(W, D, N, lam, s, z, W->X.d(), st)) return rc;
  const int nlp = 2 * ((D + 31) / 32);
  bool lp_parts = false;
  // target
  if (f.tgt == kTargetCorrGauss) {
    GemmOp tg = mm(N, D, D, W->X.d(), false, f.tparams, false, W->G.d(), -1.0);
    if (fused) {   // logp = 0.5 x . G + const from per-row partials
      tg.rp_w = W->X.d();
      tg.rp_part = W->lp_part.d();
      lp_parts = true;
    }
    FR_HIP(gemm(tg, st));
    if (!fused)
      hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(N, 4)), dim3(256), 0, st, D, (long long)N,
                         (f.chivi || f.pd) ? z : nullptr, W->X.d(), W->G.d(), f.tconst, 1,
                         W->zz.d(), W->logp.d());
  } else {
    if (int rc = eval_target(W, f.tgt, f.host, D, N, W->X.d(), W->logp.d(), W->G.d(), st)) return rc;
    if (!fused && (f.chivi || f.pd))
      hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(N, 4)), dim3(256), 0, st, D, (long long)N,
                         z, nullptr, nullptr, 0.0, 0, W->zz.d(), nullptr);
  }
  // cotangent of S: G_S = Z^T diag(r / s) G, r the objective's weights
  GemmOp g = mm(D, D, N, z, true, W->G.d(), false, W->GS.d());
  if (weights_fused() && N <= 512 && gemm_detail::glds_ok_shape(g)) {
    WeightsArgs wa{N, D, f.chivi, f.pd, f.alpha, f.df, f.t_const, W->logp.d(), W->zz.d(), s,
                   W->scal.d(), W->r.d(), W->rk.d(), value,
                   lp_parts ? W->lp_part.d() : nullptr, lp_parts ? nlp : 0, f.tconst};
    FR_HIP(gemm_hook<WeightsHook>(g, wa, st));
  } else {
    hipLaunchKernelGGL(fr_weights_kernel, dim3(1), dim3(1024), 0, st, N, D, f.chivi, f.pd, f.alpha,
                       f.df, f.t_const, W->logp.d(), W->zz.d(), s, W->scal.d(), W->r.d(),
                       W->rk.d(), value, lp_parts ? W->lp_part.d() : nullptr, lp_parts ? nlp : 0,
                       f.tconst);
    g.kscale = W->rk.d();
    FR_HIP(gemm(g, st));
  }
  if (!fused)
    hipLaunchKernelGGL(fr_colsum_kernel, dim3(blocks(D, 64)), dim3(1024), 0, st, N, D, W->r.d(),
                       W->G.d(), grad);
  // Sylvester solve (sqrtm VJP): X, symmetric Sigma cotangent of the sample term
  if (int rc = fused ? fr_pcg(W, D, st, N, W->r.d(), W->G.d(), grad) : fr_pcg(W, D, st)) return rc;
  // G_L = X L, packed with the exp-diagonal chain rule; the entropy / log q term
  // 2 c Sigma^-1 contributes 2 c Sigma^-1 L = 2 c L^-T, whose lower triangle is
  // diag(2 c / L_ii): 2 c on each packed (log) diagonal entry
  FR_HIP(gemm(mm(D, D, D, W->Xs.d(), false, W->L.d(), false, W->H.d()), st));
  const int nt = (D + kTile - 1) / kTile;
  FrSched* sc = static_cast<FrSched*>(W->sched.p);
  if (!fused) {
    hipLaunchKernelGGL(fr_pack_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, W->H.d(),
                       W->L.d(), W->scal.d(), sc, W->rr_part.d(), nt * nt, grad, W->pcg_tol2,
                       W->pcg_last);
    FR_HIP(hipGetLastError());
    return 0;
  }
  // the next step can be prepared when this root ran a Z power step (uZ valid)
  const bool prep = next && next->prep && W->last_warm && W->last_hz;
  FrPackArgs a{};
  a.D = D;
  const long long P = D + (long long)D * (D + 1) / 2;
  a.npb = (int)blocks(P);
  a.nrows = prep ? N : 0;
  a.nzb = prep ? (D + 7) / 8 : 0;
  a.GL = W->H.d();
  a.L = W->L.d();
  a.scal = W->scal.d();
  a.sc = sc;
  a.rr_part = W->rr_part.d();
  a.n_rr = nt * nt;
  a.pcg_tol2 = W->pcg_tol2;
  a.pcg_last = W->pcg_last;
  a.gmu = grad;
  a.lam = const_cast<double*>(lam);
  a.ring = up->ring;
  a.W = up->W;
  a.step = up->step;
  a.lr = up->lr;
  a.eps = up->eps;
  a.hrow = up->hrow;
  a.rng = Rng{k0, k1, stream};
  a.next_step = prep ? next->step : 0;
  a.df = f.df;
  a.z = W->Z.d();
  a.s = W->s.d();
  a.zz = W->zz.d();
  a.Zf = W->Zf;
  a.uZ = W->uZ.d();
  a.pz = W->pz.d();
  a.Sig = W->Sig.d();
  a.uS = W->uS.d();
  a.pS = W->pS.d();
  hipLaunchKernelGGL(fr_pack_update_kernel, dim3(a.npb + a.nrows + 2 * a.nzb), dim3(256), 0, st, a);
  FR_HIP(hipGetLastError());
  if (prep) {
    W->prep_owner = owner;
    W->prep_step = next->step;
    W->prep_k0 = k0;
    W->prep_k1 = k1;
    W->prep_stream = stream;
  }
  return 0;
}

// log q(x) for arbitrary x (n x D) at lam
int fr_logdensity(FrWork* W, int D, double df, double t_const, const double* lam, const double* x,
                  long long n, double* out, hipStream_t st) {
  if (int rc = fr_prepare(W, D, lam, st)) return rc;
  if (int rc = reserve_n(W, D, n)) return rc;
  hipLaunchKernelGGL(fr_center_kernel, dim3(blocks(n * D)), dim3(256), 0, st, D, n, x, lam,
                     W->X.d());
  FR_HIP(gemm(mm((int)n, D, D, W->X.d(), false, W->E.d(), true, W->G.d()), st));
  hipLaunchKernelGGL(fr_logq_kernel, dim3(blocks(n, 4)), dim3(256), 0, st, D, n, W->G.d(), W->w.d(),
                     W->scal.d(), df, t_const, out);
  FR_HIP(hipGetLastError());
  return 0;
}

// log weights lw = log p(x) - log q(x), x ~ q (experiments.py:60-63).  log q uses
// the Mahalanobis invariant z^T z / s^2.
int fr_log_weights(FrWork* W, const FrSpec& f, const double* lam, long long m,
                   const double* host_eps, uint32_t k0, uint32_t k1, uint32_t stream,
                   uint32_t step, double* lw, double* xs, hipStream_t st) {
  W->prep_owner = nullptr;
  const int D = f.D;
  if (int rc = fr_sqrt(W, D, lam, st, false)) return rc;
  if (int rc = reserve_n(W, D, m)) return rc;
  const double *s, *z;
  if (int rc = fr_draw(W, D, m, f.df, host_eps, k0, k1, stream, step, &s, &z, st)) return rc;
  double* x = xs ? xs : W->X.d();
  if (int rc = fr_transform(W, D, m, lam, s, z, x, st)) return rc;
  if (f.tgt == kTargetCorrGauss) {
    FR_HIP(gemm(mm((int)m, D, D, x, false, f.tparams, false, W->G.d(), -1.0), st));
    hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(m, 4)), dim3(256), 0, st, D, m, z, x, W->G.d(),
                       f.tconst, 1, W->zz.d(), W->logp.d());
  } else {
    if (int rc = eval_target(W, f.tgt, f.host, D, m, x, W->logp.d(), nullptr, st)) return rc;
    hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(m, 4)), dim3(256), 0, st, D, m, z, nullptr,
                       nullptr, 0.0, 0, W->zz.d(), nullptr);
  }
  // chivi weights with alpha = 1 would rescale; compute lw directly instead
  FR_HIP(launch_fr_lw(D, m, f.df, f.t_const, W->logp.d(), W->zz.d(), s, W->scal.d(), lw, st));
  return 0;
}

namespace {
__global__ __launch_bounds__(256) void fr_lw_kernel(int D, long long m, double df, double t_const,
                                                    const double* logp, const double* zz,
                                                    const double* s, const double* scal,
                                                    double* lw) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= m) return;
  const double maha = zz[k] / (s[k] * s[k]);
  const double logq = (t_const - scal[0]) - 0.5 * (df + D) * log(1.0 + maha / df);
  lw[k] = logp[k] - logq;
}
}  // namespace

hipError_t launch_fr_lw(int D, long long m, double df, double t_const, const double* logp,
                        const double* zz, const double* s, const double* scal, double* lw,
                        hipStream_t st) {
  hipLaunchKernelGGL(fr_lw_kernel, dim3(blocks(m)), dim3(256), 0, st, D, m, df, t_const, logp, zz,
                     s, scal, lw);
  return hipGetLastError();
}

// ---- mean-field families at any D with any objective / target ---------------
// The materialised path: x [N][D] is written once, the target evaluated by rows,
// per-sample weights formed, and the gradient reduced column by column.  Used
// where the fused column-pair kernel does not apply (CHIVI, whose weights couple
// all coordinates of a sample, and non-separable targets) for D > kBlockDMax.
namespace {

// KLVI: value = -(entropy + mean logp), r_n = -1/N, rsum = -1 (the entropy's
// d/dlog sigma).  CHIVI: lw = logp - logq, w = exp(lw - max)^alpha,
// value = log(mean w)/alpha + max, r_n = alpha w_n / N, rsum = sum_n r_n.
// logp / logq hold nparts partials per row ([part][N], summed in part order).
__device__ __forceinline__ double parts_sum(const double* p, int nparts, int N, int k) {
  double a = p[k];
  for (int c = 1; c < nparts; ++c) a += p[(long long)c * N + k];
  return a;
}

__global__ __launch_bounds__(1024) void mfw_weights_kernel(int N, int D, int chivi, int pd,
                                                           double alpha,
                                                           double c0, const double* lam,
                                                           const double* logp,
                                                           const double* logq, int nparts,
                                                           double* r, double* scal,
                                                           double* value) {
  __shared__ double red[16];
  // stage the chunk partials in LDS first: many independent loads in flight
  // instead of each thread's chain of nparts dependent global round trips
  constexpr int kPartsLds = 6144;
  __shared__ double s_parts[kPartsLds];
  const int pn = nparts * N;
  if (nparts > 1 && 2LL * pn <= kPartsLds) {
    const bool lq = chivi || pd;
#pragma unroll 4
    for (int i = threadIdx.x; i < pn; i += blockDim.x) {
      s_parts[i] = logp[i];
      s_parts[pn + i] = lq ? logq[i] : 0.0;
    }
    __syncthreads();
    logp = s_parts;
    logq = s_parts + pn;
  }
  if (!chivi) {
    double a = 0.0, e = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      const double lpk = parts_sum(logp, nparts, N, k);
      a += pd ? lpk - parts_sum(logq, nparts, N, k) : lpk;  // black_box_klvi_pd: sampled log q
      r[k] = -1.0 / N;
    }
    for (int d = threadIdx.x; d < D; d += blockDim.x) e += lam[D + d];
    a = block_sum(a, red);
    e = block_sum(e, red);
    if (threadIdx.x == 0) {
      *value = pd ? -(a / N) : -((c0 + e) + a / N);
      scal[1] = -1.0;
    }
    return;
  }
  double mx = -INFINITY, sw = 0.0;
  if (N <= (int)blockDim.x) {  // one row per thread: log weights stay in registers
    const int k = threadIdx.x;
    const double lw =
        k < N ? parts_sum(logp, nparts, N, k) - parts_sum(logq, nparts, N, k) : -INFINITY;
    mx = block_max(lw, red);
    const double w = k < N ? pow(exp(lw - mx), alpha) : 0.0;
    if (k < N) r[k] = alpha * w / N;
    sw = block_sum(w, red);
  } else {
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      const double lw = parts_sum(logp, nparts, N, k) - parts_sum(logq, nparts, N, k);
      r[k] = lw;
      mx = fmax(mx, lw);
    }
    mx = block_max(mx, red);
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      const double w = pow(exp(r[k] - mx), alpha);
      sw += w;
      r[k] = alpha * w / N;
    }
    sw = block_sum(sw, red);
  }
  if (threadIdx.x == 0) {
    *value = log(sw / N) / alpha + mx;
    scal[1] = alpha * sw / N;
  }
}

// grad_mu_j = sum_n r_n G_nj;  grad_logsigma_j = sigma_j sum_n r_n G_nj z_nj + rsum,
// z = (x - mu) / sigma (the standardized draw).  kGradWaves waves split the rows
// (enough waves in flight to stream X and G with N ~ 100 rows per column);
// partial sums combined in a fixed order.
//
// WFUSE (CHIVI, N <= 1024): every block first recomputes the CHIVI weights of
// mfw_weights_kernel from the per-row log p / log q partials (staged in LDS; the
// same expressions, so r and rsum are bitwise those of the separate kernel) and
// block 0 writes the value: one launch fewer per step.
// UPD: apply the windowed adagrad step to the block's columns right after their
// gradient (adagrad_step, as adagrad_update_kernel) and copy the new parameters
// to the history row: two launches fewer.  Safe because a block reads and
// writes only its own columns of lam.
constexpr int kGradWaves = 16;
constexpr int kGradLds = 6144;  // doubles: chunk-partial staging, then pa / pb

struct MfwGradArgs {
  int N, D, nparts;
  double alpha;
  double* lam;
  const double *X, *G, *r, *scal, *logp, *logq;
  double *grad, *value;
  double* ring;  // UPD
  int W;
  long long step;
  double lr, eps;
  double* hrow;  // nullable
};

template <bool WFUSE, bool UPD>
__global__ __launch_bounds__(64 * kGradWaves) void mfw_grad_kernel(MfwGradArgs A) {
  __shared__ double buf[kGradLds];
  __shared__ double s_r[WFUSE ? 1024 : 1];
  __shared__ double red[16];
  const int N = A.N, D = A.D;
  const double* r = A.r;
  double rsum;
  if constexpr (WFUSE) {
    const int k = threadIdx.x, np = A.nparts;
    double lw = -INFINITY;
    const int G = np > 1 ? min(np, 1024 / max(N, 1)) : 1;  // threads per row for the part sums
    if (G > 1) {
      // thread (g, k) sums parts g, g + G, ... of row k (logp and logq) into LDS;
      // then row k adds its G group sums in group order.  Independent loads, short
      // chains: the per-row chain of 2 * nparts dependent loads was the long pole.
      const int g = k / N, kk = k - g * N;
      if (g < G) {
        double a = 0.0, b = 0.0;
#pragma unroll 4
        for (int c = g; c < np; c += G) {
          a += A.logp[(long long)c * N + kk];
          b += A.logq[(long long)c * N + kk];
        }
        buf[g * N + kk] = a;
        buf[(G + g) * N + kk] = b;
      }
      __syncthreads();
      if (k < N) {
        double a = buf[k], b = buf[G * N + k];
        for (int q = 1; q < G; ++q) {
          a += buf[q * N + k];
          b += buf[(G + q) * N + k];
        }
        lw = a - b;
      }
    } else if (k < N) {
      lw = parts_sum(A.logp, np, N, k) - parts_sum(A.logq, np, N, k);
    }
    const int nw = (N + 63) >> 6, wave = k >> 6;  // waves holding rows
    double m = wave_max_dpp(lw);
    if ((k & 63) == 0) red[wave] = m;
    __syncthreads();
    double mx = red[0];
    for (int q = 1; q < nw; ++q) mx = fmax(mx, red[q]);
    const double w = k < N ? pow(exp(lw - mx), A.alpha) : 0.0;
    if (k < N) s_r[k] = A.alpha * w / N;
    const double ws = wave_sum_dpp(w);
    __syncthreads();
    if ((k & 63) == 0) red[wave] = ws;
    __syncthreads();  // also publishes s_r and frees buf for pa / pb
    double sw = red[0];
    for (int q = 1; q < nw; ++q) sw += red[q];
    rsum = A.alpha * sw / N;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *A.value = log(sw / N) / A.alpha + mx;
    }
    r = s_r;
  } else {
    rsum = A.scal[1];
  }
  double(*pa)[64] = reinterpret_cast<double(*)[64]>(buf);
  double(*pb)[64] = reinterpret_cast<double(*)[64]>(buf + kGradWaves * 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  double a = 0.0, b = 0.0;
  if (j < D) {
    const double mu = A.lam[j], sg = exp(A.lam[D + j]);
    for (int n = wv; n < N; n += kGradWaves) {
      const double g = r[n] * A.G[(long long)n * D + j];
      a += g;
      b += g * ((A.X[(long long)n * D + j] - mu) / sg);
    }
  }
  pa[wv][lane] = a;
  pb[wv][lane] = b;
  __syncthreads();
  if (wv == 0 && j < D) {
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int q = 0; q < kGradWaves; ++q) {
      sa += pa[q][lane];
      sb += pb[q][lane];
    }
    const double ls = A.lam[D + j];
    const double gm = sa, gs = exp(ls) * sb + rsum;
    A.grad[j] = gm;
    A.grad[D + j] = gs;
    if constexpr (UPD) {
      const long long P = 2LL * D;
      const double nm = adagrad_step(j, P, A.lam[j], gm, A.ring, A.W, A.step, A.lr, A.eps, nullptr);
      const double ns = adagrad_step(D + j, P, ls, gs, A.ring, A.W, A.step, A.lr, A.eps, nullptr);
      A.lam[j] = nm;
      A.lam[D + j] = ns;
      if (A.hrow) {
        A.hrow[j] = nm;
        A.hrow[D + j] = ns;
      }
    }
  }
}

}  // namespace

int mf_wide_value_grad(FrWork* W, const MfSpec& f, const double* lam, const double* host_eps,
                       uint32_t k0, uint32_t k1, uint32_t stream, uint32_t step, double* value,
                       double* grad, hipStream_t st, const MfUpdate* up) {
  W->prep_owner = nullptr;
  const int D = f.D, N = f.N;
  if (int rc = reserve_d(W, 1, st)) return rc;
  if (int rc = reserve_n(W, D, N)) return rc;
  if (f.tgt == kTargetCorrGauss)
    return vb_set_error(-4, "corr_gauss is implemented for the full-rank family only");
  // per-row log p / log q: one value per row, or chunk partials of the fused kernel (in Z,
  // unused on this path: nparts * N * 2 <= N * D for D >= 512)
  int nparts = 1;
  double *lp = W->logp.d(), *lq = W->zz.d();
  if (mfw_rows_fusable(f.tgt, D, N)) {
    nparts = mfw_rows_parts(D);
    lp = W->Z.d();
    lq = lp + (size_t)nparts * N;
    FR_HIP(launch_mfw_rows(f.fam, f.tgt, D, N, lam, f.t_scale, f.shape, f.df, f.t_const,
                           f.chivi || f.pd, host_eps, k0, k1, stream, step, W->X.d(), W->G.d(),
                           lp, lq, st));
  } else {
    FR_HIP(launch_sample(f.fam, D, N, lam, f.t_scale, f.shape, host_eps, k0, k1, stream, step,
                         W->X.d(), st));
    if (int rc = eval_target(W, f.tgt, f.host, D, N, W->X.d(), W->logp.d(), W->G.d(), st))
      return rc;
    if (f.chivi || f.pd)
      FR_HIP(launch_family_logdensity(f.fam, D, N, lam, f.df, f.t_const, W->X.d(), W->zz.d(), st));
  }
  const double c0 = f.fam == 1 ? 0.0 : 0.5 * D * (1.0 + kLog2Pi);
  const bool wfuse = f.chivi && N <= 1024;
  if (!wfuse)
    hipLaunchKernelGGL(mfw_weights_kernel, dim3(1), dim3(1024), 0, st, N, D, f.chivi, f.pd,
                       f.alpha, c0, lam, lp, lq, nparts, W->r.d(), W->scal.d(), value);
  MfwGradArgs A{};
  A.N = N;
  A.D = D;
  A.nparts = nparts;
  A.alpha = f.alpha;
  A.lam = const_cast<double*>(lam);  // written only with an update (the caller's parameters)
  A.X = W->X.d();
  A.G = W->G.d();
  A.r = W->r.d();
  A.scal = W->scal.d();
  A.logp = lp;
  A.logq = lq;
  A.grad = grad;
  A.value = value;
  if (up) {
    A.ring = up->ring;
    A.W = up->W;
    A.step = up->step;
    A.lr = up->lr;
    A.eps = up->eps;
    A.hrow = up->hrow;
  }
  const dim3 gg(blocks(D, 64)), gb(64 * kGradWaves);
  if (wfuse && up)
    hipLaunchKernelGGL((mfw_grad_kernel<true, true>), gg, gb, 0, st, A);
  else if (wfuse)
    hipLaunchKernelGGL((mfw_grad_kernel<true, false>), gg, gb, 0, st, A);
  else if (up)
    hipLaunchKernelGGL((mfw_grad_kernel<false, true>), gg, gb, 0, st, A);
  else
    hipLaunchKernelGGL((mfw_grad_kernel<false, false>), gg, gb, 0, st, A);
  FR_HIP(hipGetLastError());
  return 0;
}

namespace {
__global__ __launch_bounds__(256) void sub_kernel(long long n, const double* a, const double* b,
                                                  double* out) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k < n) out[k] = a[k] - b[k];
}
}  // namespace

// lw = log p(x) - log q(x), x ~ q, for any mean-field family / target / D
int mf_wide_log_weights(FrWork* W, const MfSpec& f, const double* lam, long long m,
                        const double* host_eps, uint32_t k0, uint32_t k1, uint32_t stream,
                        uint32_t step, double* lw, double* xs, hipStream_t st) {
  W->prep_owner = nullptr;
  const int D = f.D;
  if (int rc = reserve_d(W, 1, st)) return rc;
  if (int rc = reserve_n(W, D, m)) return rc;
  double* x = xs ? xs : W->X.d();
  if (f.fam == 1 && !host_eps) {
    // the t family's Philox log-weight draws are Bailey pairs (as logw_row_kernel)
    FR_HIP(launch_sample_bailey(D, m, lam, f.df, k0, k1, stream, step, x, st));
  } else {
    FR_HIP(launch_sample(f.fam, D, m, lam, f.t_scale, f.shape, host_eps, k0, k1, stream, step, x,
                         st));
  }
  if (int rc = eval_target(W, f.tgt, f.host, D, m, x, W->logp.d(), nullptr, st)) return rc;
  FR_HIP(launch_family_logdensity(f.fam, D, m, lam, f.df, f.t_const, x, W->zz.d(), st));
  hipLaunchKernelGGL(sub_kernel, dim3(blocks(m)), dim3(256), 0, st, m, W->logp.d(), W->zz.d(), lw);
  FR_HIP(hipGetLastError());
  return 0;
}

// Sigma [D][D] (nullable) and ascending eigenvalues [D] (nullable) of Sigma = L L^T
int fr_moments(FrWork* W, int D, const double* lam, double* sigma, double* eig, hipStream_t st) {
  W->prep_owner = nullptr;
  if (int rc = reserve_d(W, D, st)) return rc;
  hipLaunchKernelGGL(fr_unpack_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, lam,
                     W->L.d());
  if (sigma) FR_HIP(gemm(mm(D, D, D, W->L.d(), false, W->L.d(), true, sigma), st));
  if (eig) {
    if (int rc = fr_prepare(W, D, lam, st)) return rc;
    FR_HIP(hipMemcpyAsync(eig, W->w.d(), sizeof(double) * D, hipMemcpyDeviceToDevice, st));
  }
  return 0;
}

// Snapshot of the warm state a run's next advance starts from (its first step
// reads the previous root Z, the power vectors and the schedule block), taken on
// the stream before the advance; fr_warm_restore puts it back, so a rerun
// (vb_run_advance after a short warm root) starts from the same state as the
// failed pass did, not from where that pass ended.
int fr_warm_save(FrWork* W, hipStream_t st) {
  W->wsnap_h = FrWork::WarmHost{W->warm, W->have_z, W->zv_init, W->last_hz, false, W->pv_cur, -1,
                                W->c_slot, W->owner};
  if (W->D == 0 || !W->sched.p) return 0;   // nothing warm yet: the first step is cold
  const size_t D = (size_t)W->D, vec = sizeof(double) * D;
  FR_HIP(W->wsnap.reserve(6 * vec + vec * D + sizeof(FrSched)));
  char* p = static_cast<char*>(W->wsnap.p);
  const FrWork::Buf* v[6] = {&W->uS, &W->uZ, &W->pv[0], &W->pv[1], &W->pv[2], &W->pv[3]};
  for (int i = 0; i < 6; ++i)
    FR_HIP(hipMemcpyAsync(p + i * vec, v[i]->p, vec, hipMemcpyDeviceToDevice, st));
  if (W->have_z && W->Zf) {
    W->wsnap_h.zf_slot = W->Zf == W->Zb[0].d() ? 0 : 1;
    FR_HIP(hipMemcpyAsync(p + 6 * vec, W->Zf, vec * D, hipMemcpyDeviceToDevice, st));
  }
  FR_HIP(hipMemcpyAsync(p + 6 * vec + vec * D, W->sched.p, sizeof(FrSched),
                        hipMemcpyDeviceToDevice, st));
  W->wsnap_h.valid = true;
  return 0;
}

void fr_retry_done(FrWork* W) {
  W->retry_kmax = W->retry_pcg = 0;
  W->retry_owner = nullptr;
}

int fr_warm_restore(FrWork* W, hipStream_t st) {
  const FrWork::WarmHost h = W->wsnap_h;
  W->warm = h.warm;
  W->have_z = h.have_z;
  W->zv_init = h.zv_init;
  W->last_hz = h.last_hz;
  W->pv_cur = h.pv_cur;
  W->c_slot = h.c_slot;
  W->owner = h.owner;
  W->prep_owner = nullptr;
  if (!h.valid) {
    W->warm = false;
    return 0;
  }
  const size_t D = (size_t)W->D, vec = sizeof(double) * D;
  const char* p = static_cast<const char*>(W->wsnap.p);
  FrWork::Buf* v[6] = {&W->uS, &W->uZ, &W->pv[0], &W->pv[1], &W->pv[2], &W->pv[3]};
  for (int i = 0; i < 6; ++i)
    FR_HIP(hipMemcpyAsync(v[i]->p, p + i * vec, vec, hipMemcpyDeviceToDevice, st));
  if (h.zf_slot >= 0) {
    W->Zf = W->Zb[h.zf_slot].d();
    FR_HIP(hipMemcpyAsync(W->Zb[h.zf_slot].p, p + 6 * vec, vec * D, hipMemcpyDeviceToDevice, st));
  }
  // the schedule block, then its sticky status / hint words cleared (fr_info
  // clears them after every read-back)
  FR_HIP(hipMemcpyAsync(W->sched.p, p + 6 * vec + vec * D, sizeof(FrSched),
                        hipMemcpyDeviceToDevice, st));
  FR_HIP(hipMemsetAsync(&static_cast<FrSched*>(W->sched.p)->status, 0, 5 * sizeof(int), st));
  return 0;
}

// Reads back (one synchronisation) the outcome of the device-side iterations
// since the last call: dsyevd's info, and the sticky Newton-Schulz / PCG status;
// adapts the iteration counts launched next (one spare Newton-Schulz
// iteration; PCG: the largest converged count seen, see below).
int fr_info(FrWork* W, hipStream_t st, bool* retry) {
  int info = 0;
  const bool eig = W->info.p && W->eig_pending, sq = W->sched.p && W->sqrt_pending;
  if (!eig && !sq) return 0;
  W->eig_pending = false;
  W->sqrt_pending = false;
  if (eig) FR_HIP(hipMemcpyAsync(&info, W->info.p, sizeof(int), hipMemcpyDeviceToHost, st));
  if (sq) FR_HIP(hipMemcpyAsync(W->host_sched, W->sched.p, sizeof(FrSched), hipMemcpyDeviceToHost, st));
  FR_HIP(hipStreamSynchronize(st));
  if (info) return vb_set_error(-2, "eigendecomposition of Sigma did not converge (info %d)", info);
  if (!sq) return 0;
  const FrSched& h = *W->host_sched;
  FrSched* d = static_cast<FrSched*>(W->sched.p);
  FR_HIP(hipMemsetAsync(&d->status, 0, 5 * sizeof(int), st));   // status and the hints
  const int kpcg_seen = W->kpcg_max_seen;
  W->kpcg_max_seen = 0;
  if ((h.status & 1) || (!h.ns_conv && !h.ns_fin)) {
    // warm roots launch exactly the learnt count: a step that needed more asks
    // the caller to run its call / advance again with a larger count
    if (retry && W->last_kmax < kFrNSMax) {
      *retry = true;
      W->ns_kmax = std::min(kFrNSMax, W->last_kmax + 3);
      W->retry_kmax = W->ns_kmax;   // kept through the cold first step of the rerun
      W->retry_owner = W->owner;
      W->prep_owner = nullptr;
      return 0;
    }
    return vb_set_error(-2, "Newton-Schulz square root of Sigma did not converge in %d iterations "
                            "(Sigma too ill-conditioned)", W->last_kmax);
  }
  if (h.status & 2) {
    // the PCG's iteration count grows with the preconditioned condition number
    // (2 + k + 1/k) / 4, k = cond(S): an ill-conditioned Sigma needs far more
    // than the learnt / default count -- run again with twice as many
    if (retry && kpcg_seen < kFrPcgMax) {
      *retry = true;
      W->retry_pcg = std::min(kFrPcgMax, 2 * kpcg_seen);
      W->retry_owner = W->owner;
      W->prep_owner = nullptr;
      return 0;
    }
    return vb_set_error(-2, "conjugate gradients for the sqrtm gradient did not converge in %d "
                            "iterations", kpcg_seen);
  }
  // Newton-Schulz: launch exactly the iterations the hardest warm step needed --
  // up to its final update when the finish rule ended it (the root is then in
  // the output buffer already: no detection T and no copying launch), or up to
  // the launch that detected convergence
  if (W->last_warm && std::max(h.hint_fin, h.hint_det) > 0)
    W->ns_kmax = std::min(kFrNSMax, std::max(h.hint_fin, h.hint_det));
  // PCG: the learnt count is the index of the converged iteration, so + 1
  // launches exactly the iterations the hardest warm step so far needed (a later
  // step needing one more stops one iteration short: ~10x the 1e-9 target
  // residual, far inside the 1e-7 status bar; the next advance learns it)
  if (W->last_warm && h.hint_pcg >= 0)
    W->pcg_kmax = std::min(kFrPcgMax, std::max(h.hint_pcg, h.pcg_iter) + 1);
  return 0;
}

}  // namespace vbk

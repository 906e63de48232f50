// vb_fr.hip — full-rank Student-t family on the device
// (t_variational_family, viabel/vb.py:192-233; multivariate_t_logpdf,
// viabel/_distributions.py:8-38) and its KLVI / CHIVI value + gradient
// (vb.py:236-266).
//
// lambda = [mu (D), tril(M) row-major (D(D+1)/2)], L = M with exp'd diagonal,
// Sigma = L L^T (paragami PSDSymmetricMatrixPattern).
//
// One step (D x D products on fp64 MFMA, v_mfma_f64_16x16x4_f64):
//   L <- unpack(lambda);  E <- L L^T;  (V, w) <- eigh(E)  [rocSOLVER dsyevd]
//   S = V diag(sqrt w) V^T                       (= sqrtm(Sigma), vb.py:207)
//   X = mu + (Z S) / s                           (vb.py:208, fused epilogue)
//   G = d log p / dx, log p                      (corr_gauss: G = -X P*, GEMM)
//   KLVI : r_n = -1/N,            c = -1/2       (entropy .5 log det Sigma)
//   CHIVI: r_n = alpha w_n / N,   c = +1/2 sum r (log q's -.5 log det Sigma; the
//          Mahalanobis term is invariant under the reparameterisation)
//   G_S = Z^T diag(r / s) G                       (cotangent of S)
//   autograd's sqrtm VJP solves S X + X S = G_S; in the eigenbasis
//   M = V^T G_S V, X = V [M_ij / (sqrt w_i + sqrt w_j)] V^T, and the Sigma
//   cotangent is X + c Sigma^-1.  Sigma = L L^T gives (G + G^T) L, so only the
//   symmetric part is needed: Msym = (M + M^T) / (sqrt w_i + sqrt w_j) + 2c/w_i
//   on the diagonal;  H = V Msym V^T;  G_L = H L;  grad = [sum r G, tril(G_L)
//   with the diagonal times L_ii].
#include "vb_device.hpp"
#include "vb_internal.hpp"

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <new>

namespace vbk {
using namespace vbd;

using d4 = double __attribute__((ext_vector_type(4)));

// ---- fp64 MFMA GEMM ---------------------------------------------------------
// Block tile 32x32 (4 waves, one 16x16 MFMA tile each), K staged 16 at a time
// through LDS.  v_mfma_f64_16x16x4_f64 operand maps (cdna_hip_programming.md):
// A[l&15][k=l>>4], B[k=l>>4][l&15]; C row = (l>>4) + 4 r, col = l&15.
constexpr int kGT = 32;
constexpr int kGK = 16;

template <bool TA, bool TB, bool KS>
__global__ __launch_bounds__(256) void gemm_f64_kernel(GemmOp g) {
  __shared__ double As[kGK][kGT + 1];
  __shared__ double Bs[kGK][kGT + 1];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int i0 = blockIdx.y * kGT, j0 = blockIdx.x * kGT;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < g.K; k0 += kGK) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int idx = t + 256 * e;
      const int ia = TA ? idx % kGT : idx / kGK;
      const int ka = TA ? idx / kGT : idx % kGK;
      const int gi = i0 + ia, gka = k0 + ka;
      double v = 0.0;
      if (gi < g.M && gka < g.K) {
        v = TA ? g.A[(long long)gka * g.lda + gi] : g.A[(long long)gi * g.lda + gka];
        if (KS) v *= g.kscale[gka];
      }
      As[ka][ia] = v;
      const int jb = TB ? idx / kGK : idx % kGT;
      const int kb = TB ? idx % kGK : idx / kGT;
      const int gj = j0 + jb, gkb = k0 + kb;
      double u = 0.0;
      if (gj < g.N && gkb < g.K)
        u = TB ? g.B[(long long)gj * g.ldb + gkb] : g.B[(long long)gkb * g.ldb + gj];
      Bs[kb][jb] = u;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kGK; kk += 4) {
      const double a = As[kk + (lane >> 4)][wm * 16 + (lane & 15)];
      const double b = Bs[kk + (lane >> 4)][wn * 16 + (lane & 15)];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int col = j0 + wn * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = i0 + wm * 16 + (lane >> 4) + 4 * r;
    if (row < g.M && col < g.N) {
      double v = g.alpha * acc[r];
      if (g.row_div) v = v / g.row_div[row];
      if (g.col_bias) v = g.col_bias[col] + v;
      double* c = g.C + (long long)row * g.ldc + col;
      if (g.beta != 0.0) v += g.beta * *c;
      *c = v;
    }
  }
}

hipError_t gemm(const GemmOp& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  const dim3 grid((unsigned)((g.N + kGT - 1) / kGT), (unsigned)((g.M + kGT - 1) / kGT));
  const bool ks = g.kscale != nullptr;
#define VB_GEMM(TA, TB, KS) \
  hipLaunchKernelGGL((gemm_f64_kernel<TA, TB, KS>), grid, dim3(256), 0, s, g)
  if (!g.ta && !g.tb) { if (ks) VB_GEMM(false, false, true); else VB_GEMM(false, false, false); }
  else if (!g.ta && g.tb) { if (ks) VB_GEMM(false, true, true); else VB_GEMM(false, true, false); }
  else if (g.ta && !g.tb) { if (ks) VB_GEMM(true, false, true); else VB_GEMM(true, false, false); }
  else { if (ks) VB_GEMM(true, true, true); else VB_GEMM(true, true, false); }
#undef VB_GEMM
  return hipGetLastError();
}

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

// sq[k] = sqrt(w_k); T[k][j] = sq[k] * Vt[k][j]
__global__ __launch_bounds__(256) void fr_scale_rows_kernel(int D, const double* w,
                                                            const double* Vt, double* sq,
                                                            double* T) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)D * D) return;
  const int k = (int)(idx / D);
  const double r = sqrt(w[k]);
  T[idx] = r * Vt[idx];
  if (idx % D == 0) sq[k] = r;
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
__global__ __launch_bounds__(1024) void fr_weights_kernel(int N, int D, int chivi, double alpha,
                                                          double df, double t_const,
                                                          const double* logp, const double* zz,
                                                          const double* s, double* scal,
                                                          double* r, double* rk, double* value) {
  __shared__ double red[16];
  const double hld = scal[0];
  if (!chivi) {
    double a = 0.0;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
      a += logp[k];
      r[k] = -1.0 / N;
      rk[k] = (-1.0 / N) / s[k];
    }
    a = block_sum(a, red);
    if (threadIdx.x == 0) {
      *value = -(hld + a / N);
      scal[1] = -0.5;
    }
    return;
  }
  const double e = 0.5 * (df + D);
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

// gmu[j] = sum_n r_n G[n][j]
__global__ __launch_bounds__(256) void fr_colsum_kernel(int N, int D, const double* r,
                                                        const double* G, double* out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= D) return;
  double a = 0.0;
  for (int n = 0; n < N; ++n) a += r[n] * G[(long long)n * D + j];
  out[j] = a;
}

// Msym_ij = (M_ij + M_ji) / (sq_i + sq_j) + [i == j] 2 c / w_i
__global__ __launch_bounds__(256) void fr_sylv_kernel(int D, const double* M, const double* sq,
                                                      const double* w, const double* scal,
                                                      double* out) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)D * D) return;
  const int i = (int)(idx / D), j = (int)(idx % D);
  double v = (M[idx] + M[(long long)j * D + i]) / (sq[i] + sq[j]);
  if (i == j) v += 2.0 * scal[1] / w[i];
  out[idx] = v;
}

// grad[D + i(i+1)/2 + j] = G_L[i][j] (j < i), G_L[i][i] * L[i][i] (exp on the diagonal)
__global__ __launch_bounds__(256) void fr_pack_kernel(int D, const double* GL, const double* L,
                                                      double* grad) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long long)D * D) return;
  const int i = (int)(idx / D), j = (int)(idx % D);
  if (j > i) return;
  double v = GL[idx];
  if (j == i) v *= L[idx];
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
  Buf L, E, T, S, GS, M, H;
  // D
  Buf w, sq, offd, scal;
  Buf info;
  // N x D / N
  Buf Z, X, G, s, logp, zz, r, rk;
  long long cap_n = 0;
  ~FrWork() {
    if (blas) rocblas_destroy_handle(blas);
  }
};

FrWork* fr_work_create() { return new (std::nothrow) FrWork(); }
void fr_work_destroy(FrWork* w) { delete w; }

namespace {

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
  for (FrWork::Buf* b : {&W->L, &W->E, &W->T, &W->S, &W->GS, &W->M, &W->H}) FR_HIP(b->reserve(dd));
  for (FrWork::Buf* b : {&W->w, &W->sq, &W->offd}) FR_HIP(b->reserve(sizeof(double) * D));
  FR_HIP(W->scal.reserve(sizeof(double) * 8));
  FR_HIP(W->info.reserve(sizeof(int) * 4));
  W->D = D;
  return 0;
}

int reserve_n(FrWork* W, int D, long long n) {
  const size_t nd = sizeof(double) * (size_t)n * D, n1 = sizeof(double) * (size_t)std::max(n, 1LL);
  FR_HIP(W->Z.reserve(nd));
  FR_HIP(W->X.reserve(nd));
  FR_HIP(W->G.reserve(nd));
  for (FrWork::Buf* b : {&W->s, &W->logp, &W->zz, &W->r, &W->rk}) FR_HIP(b->reserve(n1));
  return 0;
}

}  // namespace

// L, eigh(L L^T) -> (w ascending, Vt rows = eigenvectors), half log det, S = sqrtm(Sigma)
int fr_prepare(FrWork* W, int D, const double* lam, bool need_sqrt, hipStream_t st) {
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
  hipLaunchKernelGGL(fr_logdet_kernel, dim3(1), dim3(1024), 0, st, D, W->w.d(), W->scal.d());
  if (need_sqrt) {
    hipLaunchKernelGGL(fr_scale_rows_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D,
                       W->w.d(), W->E.d(), W->sq.d(), W->T.d());
    FR_HIP(gemm(mm(D, D, D, W->E.d(), true, W->T.d(), false, W->S.d()), st));
  }
  FR_HIP(hipGetLastError());
  return 0;
}

// s (n) and z (n x D) into the workspace; host_eps = [s (n), z (n x D)] on the device
int fr_draw(FrWork* W, int D, long long n, double df, const double* host_eps, uint32_t k0,
            uint32_t k1, uint32_t stream, uint32_t step, const double** s_out,
            const double** z_out, hipStream_t st) {
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

// x = mu + (z S) / s  (after fr_prepare with need_sqrt)
int fr_transform(FrWork* W, int D, long long n, const double* mu, const double* s,
                 const double* z, double* x, hipStream_t st) {
  GemmOp g = mm((int)n, D, D, z, false, W->S.d(), false, x);
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
                  double* grad, hipStream_t st) {
  const int D = f.D, N = f.N;
  if (int rc = fr_prepare(W, D, lam, true, st)) return rc;
  if (int rc = reserve_n(W, D, N)) return rc;
  const double *s, *z;
  if (int rc = fr_draw(W, D, N, f.df, host_eps, k0, k1, stream, step, &s, &z, st)) return rc;
  if (int rc = fr_transform(W, D, N, lam, s, z, W->X.d(), st)) return rc;
  // target
  if (f.tgt == kTargetCorrGauss) {
    FR_HIP(gemm(mm(N, D, D, W->X.d(), false, f.tparams, false, W->G.d(), -1.0), st));
    hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(N, 4)), dim3(256), 0, st, D, (long long)N,
                       f.chivi ? z : nullptr, W->X.d(), W->G.d(), f.tconst, 1, W->zz.d(),
                       W->logp.d());
  } else {
    FR_HIP(launch_target_logdensity(f.tgt, D, N, W->X.d(), W->logp.d(), W->G.d(), st));
    if (f.chivi)
      hipLaunchKernelGGL(fr_rows_kernel, dim3(blocks(N, 4)), dim3(256), 0, st, D, (long long)N,
                         z, nullptr, nullptr, 0.0, 0, W->zz.d(), nullptr);
  }
  hipLaunchKernelGGL(fr_weights_kernel, dim3(1), dim3(1024), 0, st, N, D, f.chivi, f.alpha, f.df,
                     f.t_const, W->logp.d(), W->zz.d(), s, W->scal.d(), W->r.d(), W->rk.d(),
                     value);
  // cotangent of S: G_S = Z^T diag(r / s) G
  GemmOp g = mm(D, D, N, z, true, W->G.d(), false, W->GS.d());
  g.kscale = W->rk.d();
  FR_HIP(gemm(g, st));
  hipLaunchKernelGGL(fr_colsum_kernel, dim3(blocks(D)), dim3(256), 0, st, N, D, W->r.d(), W->G.d(),
                     grad);
  // Sylvester solve in the eigenbasis (Vt = E rows)
  FR_HIP(gemm(mm(D, D, D, W->E.d(), false, W->GS.d(), false, W->T.d()), st));
  FR_HIP(gemm(mm(D, D, D, W->T.d(), false, W->E.d(), true, W->M.d()), st));
  hipLaunchKernelGGL(fr_sylv_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, W->M.d(),
                     W->sq.d(), W->w.d(), W->scal.d(), W->H.d());
  FR_HIP(gemm(mm(D, D, D, W->E.d(), true, W->H.d(), false, W->T.d()), st));
  FR_HIP(gemm(mm(D, D, D, W->T.d(), false, W->E.d(), false, W->M.d()), st));
  // G_L = H L, packed with the exp-diagonal chain rule
  FR_HIP(gemm(mm(D, D, D, W->M.d(), false, W->L.d(), false, W->H.d()), st));
  hipLaunchKernelGGL(fr_pack_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, W->H.d(),
                     W->L.d(), grad);
  FR_HIP(hipGetLastError());
  return 0;
}

// log q(x) for arbitrary x (n x D) at lam
int fr_logdensity(FrWork* W, int D, double df, double t_const, const double* lam, const double* x,
                  long long n, double* out, hipStream_t st) {
  if (int rc = fr_prepare(W, D, lam, false, st)) return rc;
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
  const int D = f.D;
  if (int rc = fr_prepare(W, D, lam, true, st)) return rc;
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
    FR_HIP(launch_target_logdensity(f.tgt, D, m, x, W->logp.d(), nullptr, st));
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

// Sigma [D][D] (nullable) and ascending eigenvalues [D] (nullable) of Sigma = L L^T
int fr_moments(FrWork* W, int D, const double* lam, double* sigma, double* eig, hipStream_t st) {
  if (int rc = reserve_d(W, D, st)) return rc;
  hipLaunchKernelGGL(fr_unpack_kernel, dim3(blocks((long long)D * D)), dim3(256), 0, st, D, lam,
                     W->L.d());
  if (sigma) FR_HIP(gemm(mm(D, D, D, W->L.d(), false, W->L.d(), true, sigma), st));
  if (eig) {
    if (int rc = fr_prepare(W, D, lam, false, st)) return rc;
    FR_HIP(hipMemcpyAsync(eig, W->w.d(), sizeof(double) * D, hipMemcpyDeviceToDevice, st));
  }
  return 0;
}

int fr_info(FrWork* W, hipStream_t st) {
  int info = 0;
  if (!W->info.p) return 0;
  FR_HIP(hipMemcpyAsync(&info, W->info.p, sizeof(int), hipMemcpyDeviceToHost, st));
  FR_HIP(hipStreamSynchronize(st));
  return info;
}

}  // namespace vbk

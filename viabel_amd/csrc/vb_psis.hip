// vb_psis.hip — Pareto-smoothed importance sampling on gfx950.
//
// Reference: notebooks/psis.py (Vehtari/Sivula PSIS code)
//   psislw     psis.py:112-208
//   gpdfitnew  psis.py:211-331   (Zhang & Stephens 2009 empirical-Bayes GPD fit)
//   gpinv      psis.py:334-376
//   sumlogs    psis.py:379-395
//
// The reference sorts all n log weights (argsort) only to read ONE order
// statistic and then sorts the tail again.  Here:
//   1. max of the column (tree reduction)
//   2. radix select (8 x 8-bit digits of the order-preserving key) of the
//      element at ascending rank n - M - 1, M = ceil(min(.2n, 3 sqrt(n/Reff)))
//   3. stable compaction of x > cutoff (ascending index order, like np.where)
//   4. one-workgroup LDS bitonic sort of the tail on the key (value, position)
//      -> x2si (bit-exact tail order for distinct values)
//   5. GPD fit: one block per quadrature point b_j, then one combining block
//   6. smoothing scatter + clamp, 7. log-sum-exp renormalisation.
// All state between launches stays on the device (no host round trips), so a
// column is one stream-ordered chain of small launches.
#include "vb_device.hpp"
#include "vb_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>

using namespace vbd;

namespace vbk {

constexpr int kTailMax = 8192;  // tails up to this size: one workgroup's LDS bitonic sort;
                                // larger tails: stable device radix sort (hipcub)
constexpr int kPsisBlocks = 512;

// device scratch layout for one column (see psis_scratch_doubles)
struct PsisState {
  double mx;         // column max
  double xcut;       // cutoff
  double expcut;     // exp(cutoff)
  double k, sigma;   // GPD fit
  double lse;        // sumlogs of the smoothed column
  double b;          // posterior mean of b
  unsigned long long prefix, mask;
  long long rank;
  long long n2;      // tail size
  long long m;       // quadrature points
  long long nkeep;   // kept weights
};

__device__ __forceinline__ unsigned long long dkey(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dval(unsigned long long k) {
  const unsigned long long u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

__device__ __forceinline__ double bsum(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int q = 0; q < nw; ++q) r += red[q];
  __syncthreads();
  return r;
}
__device__ __forceinline__ double bmax(double v, double* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = -INFINITY;
  const int nw = (blockDim.x + 63) >> 6;
  for (int q = 0; q < nw; ++q) r = fmax(r, red[q]);
  __syncthreads();
  return r;
}

// ---- 1. column max -----------------------------------------------------------
__global__ __launch_bounds__(256) void col_max_kernel(const double* x, long long n, long long st,
                                                      double* part) {
  __shared__ double red[16];
  double m = -INFINITY;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    m = fmax(m, x[i * st]);
  m = bmax(m, red);
  if (threadIdx.x == 0) part[blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void max_final_kernel(const double* part, int nb, double* out) {
  __shared__ double red[16];
  double m = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += 256) m = fmax(m, part[b]);
  m = bmax(m, red);
  if (threadIdx.x == 0) *out = m;
}

// ---- 2. radix select ---------------------------------------------------------
__global__ __launch_bounds__(256) void radix_hist_kernel(const double* x, long long n,
                                                         long long st, const PsisState* ps,
                                                         int shift, unsigned* ghist) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const unsigned long long prefix = ps->prefix, mask = ps->mask;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const unsigned long long k = dkey(x[i * st]);
    if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&ghist[threadIdx.x], h[threadIdx.x]);
}

__global__ void radix_pick_kernel(const unsigned* ghist, int shift, PsisState* ps) {
  if (threadIdx.x != 0) return;
  long long r = ps->rank, cum = 0;
  int b = 0;
  for (; b < 255; ++b) {
    if (cum + (long long)ghist[b] > r) break;
    cum += ghist[b];
  }
  ps->prefix |= ((unsigned long long)b) << shift;
  ps->mask |= 255ull << shift;
  ps->rank = r - cum;
}

// cutoff = max(x_sel - max, log(tiny))  (psis.py:169-173); Python's max keeps
// the first argument unless the second is strictly greater.
__global__ void cutoff_kernel(PsisState* ps, double cutoffmin) {
  if (threadIdx.x != 0) return;
  const double xs = dval(ps->prefix) - ps->mx;
  ps->xcut = (cutoffmin > xs) ? cutoffmin : xs;
  ps->expcut = exp(ps->xcut);
}

__global__ void radix_init_kernel(PsisState* ps, long long rank) {
  if (threadIdx.x != 0) return;
  ps->prefix = 0;
  ps->mask = 0;
  ps->rank = rank;
  ps->n2 = 0;
  ps->k = NAN;
  ps->sigma = NAN;
}

// ---- 3. shift + stable compaction ------------------------------------------
__global__ __launch_bounds__(256) void shift_kernel(const double* lw, double* out, long long n,
                                                    long long st, const PsisState* ps) {
  const double mx = ps->mx;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    out[i * st] = lw[i * st] - mx;
}

__global__ __launch_bounds__(256) void tail_count_kernel(const double* x, long long n,
                                                         long long st, long long chunk,
                                                         const PsisState* ps, unsigned* cnt) {
  __shared__ unsigned wc[4];
  const double xc = ps->xcut;
  const long long r0 = (long long)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  unsigned c = 0;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256) c += (x[i * st] > xc) ? 1u : 0u;
  // wave + block sum of integers
  for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ void tail_scan_kernel(unsigned* cnt, int nb, PsisState* ps) {
  if (threadIdx.x != 0) return;
  unsigned long long acc = 0;
  for (int b = 0; b < nb; ++b) {
    const unsigned c = cnt[b];
    cnt[b] = (unsigned)acc;
    acc += c;
  }
  ps->n2 = (long long)acc;
}

__global__ __launch_bounds__(256) void tail_compact_kernel(const double* x, long long n,
                                                           long long st, long long chunk,
                                                           const PsisState* ps,
                                                           const unsigned* off, long long cap,
                                                           double* tv, long long* ti) {
  __shared__ unsigned wtot[4];
  const double xc = ps->xcut;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  unsigned base = off[blockIdx.x];
  for (long long i0 = r0; i0 < r1; i0 += 256) {
    const long long i = i0 + threadIdx.x;
    double v = 0.0;
    bool f = false;
    if (i < r1) {
      v = x[i * st];
      f = v > xc;
    }
    const unsigned long long bal = __ballot(f);
    const unsigned below = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[wid] = (unsigned)__popcll(bal);
    __syncthreads();
    unsigned wbase = 0;
    for (int q = 0; q < wid; ++q) wbase += wtot[q];
    const unsigned tot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    if (f) {
      const long long pos = (long long)base + wbase + below;
      if (pos < cap) {
        tv[pos] = v;
        ti[pos] = i;
      }
    }
    base += tot;
    __syncthreads();
  }
}

// ---- 4. bitonic sort of the tail in LDS (one workgroup) -------------------------
// Sorts (key(value), position) ascending; writes the sorted values and the
// original column indices tailinds[x2si].
__global__ __launch_bounds__(1024) void tail_sort_kernel(const double* tv, const long long* ti,
                                                         const PsisState* ps, double* sv,
                                                         long long* si, long long cap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* key = reinterpret_cast<unsigned long long*>(smem);
  unsigned* pos = reinterpret_cast<unsigned*>(smem + sizeof(unsigned long long) * kTailMax);
  if (cap > kTailMax) cap = kTailMax;
  long long n2 = ps->n2;
  if (n2 > cap) n2 = cap;
  int np2 = 1;
  while (np2 < n2) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += 1024) {
    key[i] = i < n2 ? dkey(tv[i]) : ~0ull;
    pos[i] = (unsigned)i;
  }
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const unsigned long long ki = key[i], kl = key[l];
          const unsigned pi = pos[i], pl = pos[l];
          const bool gt = (ki > kl) || (ki == kl && pi > pl);
          if (gt == up) {
            key[i] = kl;
            key[l] = ki;
            pos[i] = pl;
            pos[l] = pi;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < n2; i += 1024) {
    sv[i] = tv[pos[i]];
    si[i] = ti[pos[i]];
  }
}

// ---- 5. GPD fit (gpdfitnew, psis.py:266-331) on y = exp(sorted tail) - exp(cut)
// y[] sorted ascending, length n2 (device), or a caller array of length n.
__global__ __launch_bounds__(256) void gpd_prep_kernel(const double* sv, const PsisState* ps,
                                                       double* y, long long cap) {
  long long n2 = ps->n2;
  if (n2 > cap) n2 = cap;
  const double ec = ps->expcut;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256)
    y[i] = exp(sv[i]) - ec;
}

// one block per quadrature point j: bs[j], ks[j] = mean log1p(-b_j y)
__global__ __launch_bounds__(256) void gpd_grid_kernel(const double* y, const PsisState* ps,
                                                       long long n_fixed, double* bs,
                                                       double* ks) {
  __shared__ double red[16];
  const long long n = n_fixed > 0 ? n_fixed : ps->n2;
  if (n_fixed == 0 && n <= 4) return;  // psislw: no fit, k = inf
  const long long m = 30 + (long long)sqrt((double)n);
  const int j = blockIdx.x;
  if (j >= m) return;
  const long long q = (long long)((double)n / 4.0 + 0.5) - 1;
  // bs = 1 - sqrt(m / (j + .5)); bs /= 3 * x[q]; bs += 1 / x[-1]
  double b = 1.0 - sqrt((double)m / ((double)(j + 1) - 0.5));
  b /= 3.0 * y[q];
  b += 1.0 / y[n - 1];
  const double nb = -b;
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) s += log1p(nb * y[i]);
  s = bsum(s, red);
  if (threadIdx.x == 0) {
    bs[j] = b;
    ks[j] = s / (double)n;
  }
}

// combine: L, w, b_hat, k, sigma, prior; optional quadrature output
__global__ __launch_bounds__(256) void gpd_final_kernel(const double* y, PsisState* ps,
                                                        long long n_fixed, const double* bs,
                                                        const double* ks, double* Lw,
                                                        double* ks_out, double* w_out) {
  __shared__ double red[16];
  __shared__ double sb;
  const long long n = n_fixed > 0 ? n_fixed : ps->n2;
  if (n_fixed == 0 && n <= 4) return;
  const int m = (int)(30 + (long long)sqrt((double)n));
  double* L = Lw;
  double* w = Lw + m;
  for (int j = threadIdx.x; j < m; j += 256)
    L[j] = ((log(-(bs[j] / ks[j])) - ks[j]) - 1.0) * (double)n;
  __syncthreads();
  for (int j = threadIdx.x; j < m; j += 256) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += exp(L[i] - L[j]);
    w[j] = 1.0 / s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double thr = 10.0 * DBL_EPSILON;
    double tot = 0.0;
    long long keep = 0;
    for (int j = 0; j < m; ++j)
      if (w[j] >= thr) {
        tot += w[j];
        ++keep;
      }
    double b = 0.0;
    long long o = 0;
    for (int j = 0; j < m; ++j)
      if (w[j] >= thr) {
        const double wn = w[j] / tot;
        b += bs[j] * wn;
        if (w_out) w_out[o] = wn;
        if (ks_out) ks_out[o] = ks[j];
        ++o;
      }
    ps->nkeep = keep;
    ps->m = m;
    sb = b;
  }
  __syncthreads();
  const double b = sb;
  const double nb = -b;
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) s += log1p(nb * y[i]);
  s = bsum(s, red);
  if (threadIdx.x == 0) {
    double k = s / (double)n;
    const double sigma = -k / b * (double)n / (double)(n - 0);
    const double a = 10.0;
    k = k * (double)n / ((double)n + a) + a * 0.5 / ((double)n + a);
    ps->k = k;
    ps->sigma = sigma;
    ps->b = b;
    if (ks_out)
      for (long long o = 0; o < ps->nkeep; ++o)
        ks_out[o] = ks_out[o] * (double)n / ((double)n + a) + a * 0.5 / ((double)n + a);
  }
}

// psislw: too few tail samples -> k = inf (psis.py:177-179)
__global__ void k_inf_kernel(PsisState* ps) {
  if (threadIdx.x == 0 && ps->n2 <= 4) {
    ps->k = INFINITY;
    ps->sigma = NAN;
  }
}

// gpinv for p in (0,1) with the reference's operation order
__device__ __forceinline__ double gpinv_open(double p, double k, double sigma) {
  double x;
  if (fabs(k) < DBL_EPSILON) {
    x = -log1p(-p);
  } else {
    x = log1p(-p);
    x *= -k;
    x = expm1(x);
    x /= k;
  }
  return x * sigma;
}

// ---- 6. smoothing (psis.py:187-198) ------------------------------------------
__global__ __launch_bounds__(256) void smooth_kernel(double* x, long long st, const PsisState* ps,
                                                     const long long* si, long long cap) {
  const double k = ps->k;
  long long n2 = ps->n2;
  if (n2 > cap) n2 = cap;
  if (n2 <= 4 || !(k >= 1.0 / 3.0) || isinf(k)) return;
  const double sigma = ps->sigma, ec = ps->expcut;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (long long)gridDim.x * 256) {
    const double p = (0.5 + (double)i) / (double)n2;
    double q = (sigma <= 0.0) ? NAN : gpinv_open(p, k, sigma);
    q += ec;
    q = log(q);
    if (q > 0) q = 0.0;
    x[si[i] * st] = q;
  }
}

// ---- 7. sumlogs + renormalise -------------------------------------------------
__global__ __launch_bounds__(256) void sumexp_kernel(const double* x, long long n, long long st,
                                                     const double* mx, double* part) {
  __shared__ double red[16];
  const double m = *mx;
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    s += exp(x[i * st] - m);
  s = bsum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void lse_final_kernel(const double* part, int nb,
                                                        const double* mx, double* out) {
  __shared__ double red[16];
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[b];
  s = bsum(s, red);
  if (threadIdx.x == 0) *out = log(s) + *mx;
}

__global__ __launch_bounds__(256) void sub_kernel(double* x, long long n, long long st,
                                                  const double* v) {
  const double s = *v;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    x[i * st] -= s;
}

__global__ __launch_bounds__(256) void gpinv_kernel(const double* p, long long n, double k,
                                                    double sigma, double* out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double pi = p[i];
  double x;
  if (sigma <= 0.0) {
    x = NAN;
  } else if (pi > 0.0 && pi < 1.0) {
    x = gpinv_open(pi, k, sigma);
  } else if (pi == 0.0) {
    x = 0.0;
  } else if (pi == 1.0) {
    x = k >= 0 ? INFINITY : -sigma / k;
  } else {
    x = NAN;
  }
  out[i] = x;
}

// copy a caller array into the sort input layout (value, position)
__global__ __launch_bounds__(256) void iota_copy_kernel(const double* x, long long n, double* tv,
                                                        long long* ti, PsisState* ps) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i == 0) ps->n2 = n;
  if (i >= n) return;
  tv[i] = x[i];
  ti[i] = i;
}

// ---- host orchestration ---------------------------------------------------------
static int psis_grid(long long n) {
  long long g = (n + 2047) / 2048;
  if (g < 1) g = 1;
  if (g > kPsisBlocks) g = kPsisBlocks;
  return (int)g;
}

static size_t radix_temp_bytes(long long cap) {
  if (cap <= kTailMax) return 0;
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const double*)nullptr, (double*)nullptr,
                                           (const long long*)nullptr, (long long*)nullptr,
                                           (int)cap);
  return (bytes + 255) / 256 * 256;
}

static long long cap_of(long long cap) { return cap < kTailMax ? kTailMax : cap; }

size_t psis_scratch_bytes(long long tail_cap) {
  const long long cap = cap_of(tail_cap);
  // state + partials + radix hist + tail (value, index) x2 + y + grid arrays + sort temp
  return 256 + sizeof(double) * kPsisBlocks * 2 + sizeof(unsigned) * 256 +
         sizeof(unsigned) * kPsisBlocks + 2 * cap * (sizeof(double) + sizeof(long long)) +
         sizeof(double) * cap + sizeof(double) * 8 * 256 + radix_temp_bytes(tail_cap) + 256;
}

struct PsisScratch {
  PsisState* ps;
  double* part;
  unsigned* hist;
  unsigned* cnt;
  double* tv;
  long long* ti;
  double* sv;
  long long* si;
  double* y;
  double* bs;
  double* ks;
  double* Lw;
  void* sort_tmp;
  size_t sort_bytes;
};

static PsisScratch carve(void* base, long long tail_cap) {
  const long long kTailMax = cap_of(tail_cap);   // array capacity of this carve
  unsigned char* p = static_cast<unsigned char*>(base);
  PsisScratch s;
  s.ps = reinterpret_cast<PsisState*>(p);
  p += 256;
  s.part = reinterpret_cast<double*>(p);
  p += sizeof(double) * kPsisBlocks * 2;
  s.hist = reinterpret_cast<unsigned*>(p);
  p += sizeof(unsigned) * 256;
  s.cnt = reinterpret_cast<unsigned*>(p);
  p += sizeof(unsigned) * kPsisBlocks;
  s.tv = reinterpret_cast<double*>(p);
  p += sizeof(double) * kTailMax;
  s.ti = reinterpret_cast<long long*>(p);
  p += sizeof(long long) * kTailMax;
  s.sv = reinterpret_cast<double*>(p);
  p += sizeof(double) * kTailMax;
  s.si = reinterpret_cast<long long*>(p);
  p += sizeof(long long) * kTailMax;
  s.y = reinterpret_cast<double*>(p);
  p += sizeof(double) * kTailMax;
  s.bs = reinterpret_cast<double*>(p);
  s.ks = s.bs + 256;
  s.Lw = s.ks + 256;
  p += sizeof(double) * 8 * 256;
  p = reinterpret_cast<unsigned char*>((reinterpret_cast<uintptr_t>(p) + 255) & ~uintptr_t(255));
  s.sort_tmp = p;
  s.sort_bytes = radix_temp_bytes(tail_cap);
  return s;
}

long long psis_tail_max() { return 1LL << 30; }

namespace {
__global__ __launch_bounds__(256) void fill_inf_kernel(double* v, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = INFINITY;
}

// tail values tv / indices ti (n2 <= cap valid entries, the rest +inf when cap >
// kTailMax) -> ascending sv / si, stable on position
hipError_t sort_tail(const PsisScratch& S, long long cap, hipStream_t s) {
  if (cap <= kTailMax) {
    const size_t lds = (sizeof(unsigned long long) + sizeof(unsigned)) * kTailMax;
    hipLaunchKernelGGL(tail_sort_kernel, dim3(1), dim3(1024), lds, s, S.tv, S.ti, S.ps, S.sv, S.si,
                       cap);
    return hipGetLastError();
  }
  size_t bytes = S.sort_bytes;
  return hipcub::DeviceRadixSort::SortPairs(S.sort_tmp, bytes, S.tv, S.sv, S.ti, S.si, (int)cap, 0,
                                            64, s);
}
}  // namespace

// One column of psislw.  lw/out are device pointers with stride st.
hipError_t psis_column(const double* lw, double* out, long long n, long long st, long long Mt,
                       void* scratch, double* k_dev, long long* tail_idx_dev,
                       long long* n_tail_dev, hipStream_t s) {
  const long long cap = Mt < 1 ? 1 : Mt;   // the tail holds at most M_t draws
  PsisScratch S = carve(scratch, cap);
  const int g = psis_grid(n);
  // 1. max
  hipLaunchKernelGGL(col_max_kernel, dim3(g), dim3(256), 0, s, lw, n, st, S.part);
  hipLaunchKernelGGL(max_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->mx);
  // 2. radix select of ascending rank n - Mt - 1
  hipLaunchKernelGGL(radix_init_kernel, dim3(1), dim3(64), 0, s, S.ps, n - Mt - 1);
  hipError_t e;
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    e = hipMemsetAsync(S.hist, 0, sizeof(unsigned) * 256, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(g), dim3(256), 0, s, lw, n, st, S.ps, shift, S.hist);
    hipLaunchKernelGGL(radix_pick_kernel, dim3(1), dim3(64), 0, s, S.hist, shift, S.ps);
  }
  hipLaunchKernelGGL(cutoff_kernel, dim3(1), dim3(64), 0, s, S.ps, log(DBL_MIN));
  // 3. shifted copy + stable tail compaction
  const long long chunk = ((n + g - 1) / g + 255) / 256 * 256;
  const int gc = (int)((n + chunk - 1) / chunk);
  hipLaunchKernelGGL(shift_kernel, dim3(g), dim3(256), 0, s, lw, out, n, st, S.ps);
  hipLaunchKernelGGL(tail_count_kernel, dim3(gc), dim3(256), 0, s, out, n, st, chunk, S.ps, S.cnt);
  hipLaunchKernelGGL(tail_scan_kernel, dim3(1), dim3(64), 0, s, S.cnt, gc, S.ps);
  if (cap > kTailMax)
    hipLaunchKernelGGL(fill_inf_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, S.tv,
                       cap);
  hipLaunchKernelGGL(tail_compact_kernel, dim3(gc), dim3(256), 0, s, out, n, st, chunk, S.ps, S.cnt,
                     cap, S.tv, S.ti);
  // 4. sort the tail
  e = sort_tail(S, cap, s);
  if (e != hipSuccess) return e;
  // 5. GPD fit (skipped on device when n2 <= 4)
  hipLaunchKernelGGL(gpd_prep_kernel, dim3(32), dim3(256), 0, s, S.sv, S.ps, S.y, cap);
  const int mmax = 30 + (int)std::sqrt((double)Mt) + 1;
  hipLaunchKernelGGL(gpd_grid_kernel, dim3(mmax), dim3(256), 0, s, S.y, S.ps, 0LL, S.bs, S.ks);
  hipLaunchKernelGGL(gpd_final_kernel, dim3(1), dim3(256), 0, s, S.y, S.ps, 0LL, S.bs, S.ks, S.Lw,
                     nullptr, nullptr);
  hipLaunchKernelGGL(k_inf_kernel, dim3(1), dim3(64), 0, s, S.ps);
  // 6. smoothing
  hipLaunchKernelGGL(smooth_kernel, dim3(32), dim3(256), 0, s, out, st, S.ps, S.si, cap);
  // 7. renormalise: x -= sumlogs(x)
  hipLaunchKernelGGL(col_max_kernel, dim3(g), dim3(256), 0, s, out, n, st, S.part);
  hipLaunchKernelGGL(max_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b);
  hipLaunchKernelGGL(sumexp_kernel, dim3(g), dim3(256), 0, s, out, n, st, &S.ps->b, S.part);
  hipLaunchKernelGGL(lse_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b, &S.ps->lse);
  hipLaunchKernelGGL(sub_kernel, dim3(g), dim3(256), 0, s, out, n, st, &S.ps->lse);
  e = hipMemcpyAsync(k_dev, &S.ps->k, sizeof(double), hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  if (n_tail_dev) {
    e = hipMemcpyAsync(n_tail_dev, &S.ps->n2, sizeof(long long), hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  if (tail_idx_dev) {
    e = hipMemcpyAsync(tail_idx_dev, S.si, sizeof(long long) * Mt, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// gpdfitnew on a caller array x[n] (device), any order.  out4 = {k, sigma, m, nkeep}
hipError_t psis_gpdfit(const double* x, long long n, void* scratch, double* out4,
                       double* ks_out, double* w_out, hipStream_t s) {
  PsisScratch S = carve(scratch, n);
  hipLaunchKernelGGL(iota_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n,
                     S.tv, S.ti, S.ps);
  hipError_t e0 = sort_tail(S, n, s);
  if (e0 != hipSuccess) return e0;
  const int m = 30 + (int)std::sqrt((double)n);
  hipLaunchKernelGGL(gpd_grid_kernel, dim3(m), dim3(256), 0, s, S.sv, S.ps, n, S.bs, S.ks);
  hipLaunchKernelGGL(gpd_final_kernel, dim3(1), dim3(256), 0, s, S.sv, S.ps, n, S.bs, S.ks, S.Lw,
                     ks_out, w_out);
  hipError_t e = hipMemcpyAsync(out4, &S.ps->k, sizeof(double) * 2, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(out4 + 2, &S.ps->m, sizeof(long long) * 2, hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t psis_gpinv(const double* p, long long n, double k, double sigma, double* out,
                      hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gpinv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n, k,
                     sigma, out);
  return hipGetLastError();
}

hipError_t psis_sumlogs(const double* x, long long n, void* scratch, double* out, hipStream_t s) {
  PsisScratch S = carve(scratch, 0);
  const int g = psis_grid(n);
  hipLaunchKernelGGL(col_max_kernel, dim3(g), dim3(256), 0, s, x, n, 1LL, S.part);
  hipLaunchKernelGGL(max_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b);
  hipLaunchKernelGGL(sumexp_kernel, dim3(g), dim3(256), 0, s, x, n, 1LL, &S.ps->b, S.part);
  hipLaunchKernelGGL(lse_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b, out);
  return hipGetLastError();
}

}  // namespace vbk

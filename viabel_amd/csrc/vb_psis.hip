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
// Fast path for tails of <= kTailMax candidates (psis_columns, round 4): the
// column max and an 11-bit histogram of the key in one pass, a second 11-bit
// histogram inside the selected bin, then ONE compaction of every element whose
// 22-bit key prefix is >= the selected one (the order statistic and everything
// above it, ~M + a few dozen draws) and one LDS sort of those on (key of x - max,
// index): the order statistic, the cutoff and the sorted tail fall out of the
// sorted candidates.  3 passes over the column instead of 11; the same bits.
//   5. GPD fit: one block per quadrature point b_j, then one combining block
//   6. smoothing scatter + clamp, 7. log-sum-exp renormalisation.
// All state between launches stays on the device, so a column is one
// stream-ordered chain of small launches -- except for one host round trip on
// the fast path: after the two histogram passes the host reads the per-column
// "candidates fit" flags (into a pinned buffer, one stream wait) and launches
// either the candidate sort or the radix path.  Keeping both paths' launches
// with device-side early exits instead would add ~20 empty launches (~40 us) to
// every call; the round trip costs one wait (~10 us).  (So psis_columns cannot
// be captured into a hipGraph.)
#include "vb_device.hpp"
#include "vb_internal.hpp"

#include <algorithm>
#include <cstdlib>


#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cmath>

using namespace vbd;

namespace vbk {

constexpr int kTailMax = 8192;  // tails up to this size: one workgroup's LDS bitonic sort;
                                // larger tails: stable device radix sort (hipcub)
constexpr int kPsisBlocks = 512;

// VIABEL_AMD_PSIS_FAST_SELECT=0: always the 8-pass radix select (A/B switch; same bits)
static bool psis_fast_select_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_PSIS_FAST_SELECT");
    return !(e && e[0] == '0');
  }();
  return on;
}

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
  long long above;   // two-digit select: elements above the selected bins
  long long cand;    // candidates: elements whose 22-bit key prefix >= the selected one
  unsigned long long cnt;   // candidate compaction counter
};
static_assert(sizeof(PsisState) <= 256, "PsisState fits its scratch slot");

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

// Column batching: every per-column kernel takes its column from blockIdx.y.
// Element (i, c) of the input / output is x[c * cs + i * rs]; column c's
// scratch (PsisState, partials, tail buffers, ...) sits sb bytes after column
// c - 1's, so one launch sequence serves all m columns of a psislw call.
template <class T>
__device__ __forceinline__ T* colp(T* p, long long sb) {
  return reinterpret_cast<T*>(reinterpret_cast<unsigned char*>(p) + (long long)blockIdx.y * sb);
}
template <class T>
__device__ __forceinline__ const T* colp(const T* p, long long sb) {
  return reinterpret_cast<const T*>(reinterpret_cast<const unsigned char*>(p) +
                                    (long long)blockIdx.y * sb);
}

// ---- 1. column max -----------------------------------------------------------
__global__ __launch_bounds__(256) void col_max_kernel(const double* x, long long n, long long rs,
                                                      long long cs, double* part, long long sb) {
  __shared__ double red[16];
  x += (long long)blockIdx.y * cs;
  double m = -INFINITY;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    m = fmax(m, x[i * rs]);
  m = bmax(m, red);
  if (threadIdx.x == 0) colp(part, sb)[blockIdx.x] = m;
}

__global__ __launch_bounds__(256) void max_final_kernel(const double* part, int nb, double* out,
                                                        long long sb) {
  __shared__ double red[16];
  part = colp(part, sb);
  double m = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += 256) m = fmax(m, part[b]);
  m = bmax(m, red);
  if (threadIdx.x == 0) *colp(out, sb) = m;
}

// ---- 2. radix select ---------------------------------------------------------
__global__ __launch_bounds__(256) void radix_hist_kernel(const double* x, long long n,
                                                         long long rs, long long cs,
                                                         const PsisState* ps, int shift,
                                                         unsigned* ghist, long long sb) {
  __shared__ unsigned h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  x += (long long)blockIdx.y * cs;
  ps = colp(ps, sb);
  const unsigned long long prefix = ps->prefix, mask = ps->mask;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256) {
    const unsigned long long k = dkey(x[i * rs]);
    if ((k & mask) == prefix) atomicAdd(&h[(k >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&colp(ghist, sb)[threadIdx.x], h[threadIdx.x]);
}

// picks the digit, then clears the histogram for the next pass
__global__ __launch_bounds__(256) void radix_pick_kernel(unsigned* ghist, int shift, PsisState* ps,
                                                         long long sb) {
  __shared__ unsigned h[256];
  ghist = colp(ghist, sb);
  ps = colp(ps, sb);
  h[threadIdx.x] = ghist[threadIdx.x];
  ghist[threadIdx.x] = 0;
  __syncthreads();
  if (threadIdx.x != 0) return;
  long long r = ps->rank, cum = 0;
  int b = 0;
  for (; b < 255; ++b) {
    if (cum + (long long)h[b] > r) break;
    cum += h[b];
  }
  ps->prefix |= ((unsigned long long)b) << shift;
  ps->mask |= 255ull << shift;
  ps->rank = r - cum;
}

// cutoff = max(x_sel - max, log(tiny))  (psis.py:169-173); Python's max keeps
// the first argument unless the second is strictly greater.
__global__ void cutoff_kernel(PsisState* ps, double cutoffmin, long long sb) {
  if (threadIdx.x != 0) return;
  ps = colp(ps, sb);
  const double xs = dval(ps->prefix) - ps->mx;
  ps->xcut = (cutoffmin > xs) ? cutoffmin : xs;
  ps->expcut = exp(ps->xcut);
}

__global__ __launch_bounds__(256) void radix_init_kernel(PsisState* ps, unsigned* ghist,
                                                         long long rank, long long sb) {
  colp(ghist, sb)[threadIdx.x] = 0;
  if (threadIdx.x != 0) return;
  ps = colp(ps, sb);
  ps->prefix = 0;
  ps->mask = 0;
  ps->rank = rank;
  ps->n2 = 0;
  ps->k = NAN;
  ps->sigma = NAN;
}

// ---- 2'. two-digit select + candidate compaction (fast path) -----------------
constexpr int kSelBins = 2048;              // 11-bit digits
constexpr int kSelShift1 = 53, kSelShift2 = 42;

__global__ __launch_bounds__(256) void sel_init_kernel(PsisState* ps, unsigned* gh, long long rank,
                                                       long long sb) {
  gh = colp(gh, sb);
  for (int b = threadIdx.x; b < kSelBins; b += 256) gh[b] = 0;
  if (threadIdx.x != 0) return;
  ps = colp(ps, sb);
  ps->prefix = 0;
  ps->mask = 0;
  ps->rank = rank;
  ps->n2 = 0;
  ps->k = NAN;
  ps->sigma = NAN;
  ps->above = 0;
  ps->cand = 0;
  ps->cnt = 0;
}

// pass 1: the column max (block partials) and the histogram of the top 11 key bits
__global__ __launch_bounds__(256) void sel_hist1_kernel(const double* x, long long n, long long rs,
                                                        long long cs, double* part, unsigned* gh,
                                                        long long sb) {
  __shared__ unsigned h[kSelBins];
  __shared__ double red[16];
  for (int b = threadIdx.x; b < kSelBins; b += 256) h[b] = 0;
  __syncthreads();
  x += (long long)blockIdx.y * cs;
  double m = -INFINITY;
  // four loads in flight per thread (one at a time left the pass latency-bound)
  const long long st = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = x[(i + u * st) * rs];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m = fmax(m, v[u]);
      // the top digit of log weights sits in a few bins: the lanes sharing the
      // first lane's bin add their count with one atomic (a same-address LDS
      // atomic from many lanes serialises), the others add their own
      const unsigned b = (unsigned)(dkey(v[u]) >> kSelShift1);
      const unsigned b0 = __builtin_amdgcn_readfirstlane(b);
      const unsigned long long same = __ballot(b == b0);
      if (b == b0) {
        if ((threadIdx.x & 63) == (unsigned)__builtin_ctzll(same))
          atomicAdd(&h[b0], (unsigned)__popcll(same));
      } else {
        atomicAdd(&h[b], 1u);
      }
    }
  }
  for (; i < n; i += st) {
    const double v = x[i * rs];
    m = fmax(m, v);
    atomicAdd(&h[dkey(v) >> kSelShift1], 1u);
  }
  m = bmax(m, red);   // (its barriers also complete the LDS histogram)
  if (threadIdx.x == 0) colp(part, sb)[blockIdx.x] = m;
  unsigned* g = colp(gh, sb);
  for (int b = threadIdx.x; b < kSelBins; b += 256)
    if (h[b]) atomicAdd(&g[b], h[b]);
}

// pass 2: the next 11 key bits of the elements in the selected top bin
__global__ __launch_bounds__(256) void sel_hist2_kernel(const double* x, long long n, long long rs,
                                                        long long cs, const PsisState* ps,
                                                        unsigned* gh, long long sb) {
  __shared__ unsigned h[kSelBins];
  for (int b = threadIdx.x; b < kSelBins; b += 256) h[b] = 0;
  __syncthreads();
  x += (long long)blockIdx.y * cs;
  const unsigned long long top = colp(ps, sb)->prefix >> kSelShift1;
  const long long st = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * st < n; i += 4 * st) {
    unsigned long long k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) k[u] = dkey(x[(i + u * st) * rs]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((k[u] >> kSelShift1) == top) atomicAdd(&h[(k[u] >> kSelShift2) & (kSelBins - 1)], 1u);
  }
  for (; i < n; i += st) {
    const unsigned long long k = dkey(x[i * rs]);
    if ((k >> kSelShift1) == top) atomicAdd(&h[(k >> kSelShift2) & (kSelBins - 1)], 1u);
  }
  __syncthreads();
  unsigned* g = colp(gh, sb);
  for (int b = threadIdx.x; b < kSelBins; b += 256)
    if (h[b]) atomicAdd(&g[b], h[b]);
}

// the bin holding ascending rank ps->rank of this stage's population (a parallel
// scan over 2 048 bins), then clears the histogram; stage 2 also counts the
// candidates (everything at or above the selected 22-bit prefix) and flags
// whether they fit one workgroup's sort
__global__ __launch_bounds__(256) void sel_pick_kernel(unsigned* gh, PsisState* ps, int stage,
                                                       unsigned* flag, long long sb) {
  __shared__ unsigned long long wsum[4];
  gh = colp(gh, sb);
  ps = colp(ps, sb);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned c[8];
  unsigned long long sum = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    c[k] = gh[t * 8 + k];
    sum += c[k];
  }
  unsigned long long inc = sum;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  if (lane == 63) wsum[w] = inc;
  const long long r = ps->rank;
  if (stage == 1 && t == 0) flag[blockIdx.y] = 0u;   // set by stage 2's pick
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) gh[t * 8 + k] = 0;
  unsigned long long base = 0;
  for (int q = 0; q < w; ++q) base += wsum[q];
  const unsigned long long tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const unsigned long long excl = base + inc - sum;
  if ((long long)excl <= r && r < (long long)(excl + sum)) {   // exactly one thread
    unsigned long long cum = excl;
    int b = 0;
    for (; b < 7; ++b) {
      if ((long long)(cum + c[b]) > r) break;
      cum += c[b];
    }
    const int shift = stage == 1 ? kSelShift1 : kSelShift2;
    ps->prefix |= (unsigned long long)(t * 8 + b) << shift;
    ps->mask |= (unsigned long long)(kSelBins - 1) << shift;
    ps->rank = r - (long long)cum;
    const long long above = (long long)(tot - cum - c[b]);
    if (stage == 1) {
      ps->above = above;
    } else {
      ps->above += above;
      ps->cand = ps->above + (long long)c[b];
      flag[blockIdx.y] = ps->cand <= kTailMax ? 1u : 0u;
    }
  }
}

// every element whose 22-bit key prefix is >= the selected one: (x - max, index),
// in any order (the sort orders them).  Each wave gathers its hits in LDS (ballot
// offsets, no atomics), then the block reserves its run with ONE counter add
// (a fetch-add per hit wave waited a round trip each: 378 us for the pass);
// hits past a wave's LDS capacity go out directly with a wave-level add.
constexpr int kCompactWaveCap = 128;
__global__ __launch_bounds__(256) void sel_compact_kernel(const double* x, long long n, long long rs,
                                                          long long cs, PsisState* ps, double* tv,
                                                          long long* ti, long long sb) {
  __shared__ double s_v[4][kCompactWaveCap];
  __shared__ unsigned s_i[4][kCompactWaveCap];
  __shared__ unsigned s_c[4];
  __shared__ unsigned long long s_base;
  ps = colp(ps, sb);
  if (ps->cand > kTailMax) return;
  const unsigned long long p22 = ps->prefix >> kSelShift2;
  const double mx = ps->mx;
  x += (long long)blockIdx.y * cs;
  tv = colp(tv, sb);
  ti = colp(ti, sb);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned c = 0;   // this wave's hits so far (wave-uniform)
  auto hit = [&](bool f, double v, long long i) __attribute__((always_inline)) {
    const unsigned long long bal = __ballot(f);
    if (!bal) return;
    const unsigned pos = c + (unsigned)__popcll(bal & lt);
    if (f && pos < (unsigned)kCompactWaveCap) {
      s_v[w][pos] = v;
      s_i[w][pos] = (unsigned)i;
    }
    const unsigned long long over = __ballot(f && pos >= (unsigned)kCompactWaveCap);
    if (over) {
      unsigned long long b0 = 0;
      if (lane == 0) b0 = atomicAdd(&ps->cnt, (unsigned long long)__popcll(over));
      b0 = __shfl(b0, 0, 64);
      if (f && pos >= (unsigned)kCompactWaveCap) {
        const unsigned long long q = b0 + __popcll(over & lt);
        if (q < (unsigned long long)kTailMax) {
          tv[q] = v;
          ti[q] = i;
        }
      }
    }
    c += (unsigned)__popcll(bal);
  };
  const long long st = (long long)gridDim.x * 256;
  long long i0 = (long long)blockIdx.x * 256;
  for (; i0 + 3 * st + 255 < n; i0 += 4 * st) {   // four loads in flight (all in range)
    double xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) xv[u] = x[(i0 + u * st + threadIdx.x) * rs];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      hit((dkey(xv[u]) >> kSelShift2) >= p22, xv[u] - mx, i0 + u * st + threadIdx.x);
  }
  for (; i0 < n; i0 += st) {
    const long long i = i0 + threadIdx.x;
    bool f = false;
    double v = 0.0;
    if (i < n) {
      const double xv = x[i * rs];
      f = (dkey(xv) >> kSelShift2) >= p22;
      v = xv - mx;
    }
    hit(f, v, i);
  }
  const unsigned mine = c < (unsigned)kCompactWaveCap ? c : (unsigned)kCompactWaveCap;
  if (lane == 0) s_c[w] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tot = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    s_base = tot ? atomicAdd(&ps->cnt, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  unsigned long long b = s_base;
  for (int q = 0; q < w; ++q) b += s_c[q];
  for (unsigned k = lane; k < mine; k += 64) {
    const unsigned long long q = b + k;
    if (q < (unsigned long long)kTailMax) {
      tv[q] = s_v[w][k];
      ti[q] = s_i[w][k];
    }
  }
}

// one workgroup per column: the candidates sorted on (key of x - max, index); the
// order statistic at ascending rank n - Mt - 1 is candidate (n - Mt - 1) - (n - cand);
// cutoff = max(its value, log(tiny)) as cutoff_kernel; the tail (x - max > cutoff)
// is a run of the sorted candidates, written like tail_sort_kernel's output
__global__ __launch_bounds__(1024) void sel_sort_kernel(const double* tv, const long long* ti,
                                                        PsisState* ps, double* sv, long long* si,
                                                        long long n, long long Mt, double cutoffmin,
                                                        long long sb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* key = reinterpret_cast<unsigned long long*>(smem);
  unsigned* idx = reinterpret_cast<unsigned*>(smem + sizeof(unsigned long long) * kTailMax);
  __shared__ int s_first, s_cnt;
  tv = colp(tv, sb);
  ti = colp(ti, sb);
  sv = colp(sv, sb);
  si = colp(si, sb);
  ps = colp(ps, sb);
  const long long c = ps->cand;
  if (c > kTailMax) return;
  int np2 = 1;
  while (np2 < c) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += 1024) {
    key[i] = i < c ? dkey(tv[i]) : ~0ull;
    idx[i] = i < c ? (unsigned)ti[i] : 0xFFFFFFFFu;
  }
  if (threadIdx.x == 0) {
    s_first = (int)c;
    s_cnt = 0;
  }
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const unsigned long long ki = key[i], kl = key[l];
          const unsigned pi = idx[i], pl = idx[l];
          const bool gt = (ki > kl) || (ki == kl && pi > pl);
          if (gt == up) {
            key[i] = kl;
            key[l] = ki;
            idx[i] = pl;
            idx[l] = pi;
          }
        }
      }
      __syncthreads();
    }
  }
  const long long q = (n - Mt - 1) - (n - c);
  const double xs = dval(key[q]);
  const double xc = (cutoffmin > xs) ? cutoffmin : xs;
  // the tail: candidates with value > cutoff (a contiguous run: NaNs, which never
  // compare greater, sort to the ends)
  int cnt = 0, first = (int)c;
  for (int i = threadIdx.x; i < (int)c; i += 1024)
    if (dval(key[i]) > xc) {
      ++cnt;
      first = min(first, i);
    }
  atomicAdd(&s_cnt, cnt);
  atomicMin(&s_first, first);
  __syncthreads();
  const int n2 = s_cnt, t0 = s_first;
  for (int i = threadIdx.x; i < n2; i += 1024) {
    sv[i] = dval(key[t0 + i]);
    si[i] = idx[t0 + i];
  }
  if (threadIdx.x == 0) {
    ps->xcut = xc;
    ps->expcut = exp(xc);
    ps->n2 = n2;
  }
}

// ---- 3. shift + stable compaction ------------------------------------------
__global__ __launch_bounds__(256) void shift_kernel(const double* lw, double* out, long long n,
                                                    long long rs, long long cs,
                                                    const PsisState* ps, long long sb) {
  const double mx = colp(ps, sb)->mx;
  lw += (long long)blockIdx.y * cs;
  out += (long long)blockIdx.y * cs;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    out[i * rs] = lw[i * rs] - mx;
}

// x: the shifted copy lw - max (unshifted = 0), or lw itself with the shift
// applied here (unshifted = 1; the same bits: one subtraction either way)
__global__ __launch_bounds__(256) void tail_count_kernel(const double* x, long long n,
                                                         long long rs, long long cs,
                                                         long long chunk, const PsisState* ps,
                                                         unsigned* cnt, long long sb,
                                                         int unshifted) {
  __shared__ unsigned wc[4];
  const double xc = colp(ps, sb)->xcut;
  const double mx = unshifted ? colp(ps, sb)->mx : 0.0;
  x += (long long)blockIdx.y * cs;
  const long long r0 = (long long)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  unsigned c = 0;
  for (long long i = r0 + threadIdx.x; i < r1; i += 256)
    c += ((unshifted ? x[i * rs] - mx : x[i * rs]) > xc) ? 1u : 0u;
  // wave + block sum of integers
  for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) colp(cnt, sb)[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ void tail_scan_kernel(unsigned* cnt, int nb, PsisState* ps, long long sb) {
  if (threadIdx.x != 0) return;
  cnt = colp(cnt, sb);
  unsigned long long acc = 0;
  for (int b = 0; b < nb; ++b) {
    const unsigned c = cnt[b];
    cnt[b] = (unsigned)acc;
    acc += c;
  }
  colp(ps, sb)->n2 = (long long)acc;
}

__global__ __launch_bounds__(256) void tail_compact_kernel(const double* x, long long n,
                                                           long long rs, long long cs,
                                                           long long chunk, const PsisState* ps,
                                                           const unsigned* off, long long cap,
                                                           double* tv, long long* ti,
                                                           long long sb, int unshifted) {
  __shared__ unsigned wtot[4];
  const double xc = colp(ps, sb)->xcut;
  const double mx = unshifted ? colp(ps, sb)->mx : 0.0;
  x += (long long)blockIdx.y * cs;
  tv = colp(tv, sb);
  ti = colp(ti, sb);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  unsigned base = colp(off, sb)[blockIdx.x];
  for (long long i0 = r0; i0 < r1; i0 += 256) {
    const long long i = i0 + threadIdx.x;
    double v = 0.0;
    bool f = false;
    if (i < r1) {
      v = unshifted ? x[i * rs] - mx : x[i * rs];
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

// ---- 4. bitonic sort of the tail in LDS (one workgroup per column) ------------
// Sorts (key(value), position) ascending; writes the sorted values and the
// original column indices tailinds[x2si].
__global__ __launch_bounds__(1024) void tail_sort_kernel(const double* tv, const long long* ti,
                                                         const PsisState* ps, double* sv,
                                                         long long* si, long long cap,
                                                         long long sb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* key = reinterpret_cast<unsigned long long*>(smem);
  unsigned* pos = reinterpret_cast<unsigned*>(smem + sizeof(unsigned long long) * kTailMax);
  tv = colp(tv, sb);
  ti = colp(ti, sb);
  sv = colp(sv, sb);
  si = colp(si, sb);
  if (cap > kTailMax) cap = kTailMax;
  long long n2 = colp(ps, sb)->n2;
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
                                                       double* y, long long cap, long long sb) {
  ps = colp(ps, sb);
  sv = colp(sv, sb);
  y = colp(y, sb);
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
                                                       double* ks, long long sb) {
  __shared__ double red[16];
  y = colp(y, sb);
  ps = colp(ps, sb);
  bs = colp(bs, sb);
  ks = colp(ks, sb);
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
                                                        double* ks_out, double* w_out,
                                                        long long sb) {
  __shared__ double red[16];
  __shared__ double sb_hat;
  y = colp(y, sb);
  ps = colp(ps, sb);
  bs = colp(bs, sb);
  ks = colp(ks, sb);
  Lw = colp(Lw, sb);
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
    sb_hat = b;
  }
  __syncthreads();
  const double b = sb_hat;
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
__global__ void k_inf_kernel(PsisState* ps, long long sb) {
  ps = colp(ps, sb);
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
__global__ __launch_bounds__(256) void smooth_kernel(double* x, long long rs, long long cs,
                                                     const PsisState* ps, const long long* si,
                                                     long long cap, long long sb) {
  ps = colp(ps, sb);
  si = colp(si, sb);
  x += (long long)blockIdx.y * cs;
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
    x[si[i] * rs] = q;
  }
}

// ---- 7. sumlogs + renormalise -------------------------------------------------
__global__ __launch_bounds__(256) void sumexp_kernel(const double* x, long long n, long long rs,
                                                     long long cs, const double* mx,
                                                     double* part, long long sb) {
  __shared__ double red[16];
  x += (long long)blockIdx.y * cs;
  const double m = *colp(mx, sb);
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    s += exp(x[i * rs] - m);
  s = bsum(s, red);
  if (threadIdx.x == 0) colp(part, sb)[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void lse_final_kernel(const double* part, int nb,
                                                        const double* mx, double* out,
                                                        long long sb) {
  __shared__ double red[16];
  part = colp(part, sb);
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[b];
  s = bsum(s, red);
  if (threadIdx.x == 0) *colp(out, sb) = log(s) + *colp(mx, sb);
}

__global__ __launch_bounds__(256) void sub_kernel(double* x, long long n, long long rs,
                                                  long long cs, const double* v, long long sb) {
  const double s = *colp(v, sb);
  x += (long long)blockIdx.y * cs;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (long long)gridDim.x * 256)
    x[i * rs] -= s;
}

// per-column results out of the scratch: k[c], n_tail[c], tail indices row c
__global__ __launch_bounds__(256) void psis_out_kernel(const PsisState* ps, const long long* si,
                                                       long long Mt, double* k_out,
                                                       long long* n_tail_out, long long* tail_out,
                                                       long long tail_cap, long long sb) {
  const int c = blockIdx.y;
  ps = colp(ps, sb);
  si = colp(si, sb);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    k_out[c] = ps->k;
    if (n_tail_out) n_tail_out[c] = ps->n2;
  }
  if (tail_out)
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < Mt;
         i += (long long)gridDim.x * 256)
      tail_out[(long long)c * tail_cap + i] = si[i];
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
  return 256 + sizeof(double) * kPsisBlocks * 2 + sizeof(unsigned) * kSelBins +
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
  p += sizeof(unsigned) * kSelBins;   // (the radix passes use the first 256)
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
__global__ __launch_bounds__(256) void fill_inf_kernel(double* v, long long n, long long sb) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) colp(v, sb)[i] = INFINITY;
}

template <class T>
T* offset_bytes(T* p, long long b) {
  return reinterpret_cast<T*>(reinterpret_cast<unsigned char*>(p) + b);
}

// tail values tv / indices ti (n2 <= cap valid entries, the rest +inf when cap >
// kTailMax) -> ascending sv / si, stable on position; m columns sb bytes apart
hipError_t sort_tail(const PsisScratch& S, long long cap, int m, long long sb, hipStream_t s) {
  if (cap <= kTailMax) {
    const size_t lds = (sizeof(unsigned long long) + sizeof(unsigned)) * kTailMax;
    hipLaunchKernelGGL(tail_sort_kernel, dim3(1, m), dim3(1024), lds, s, S.tv, S.ti, S.ps, S.sv,
                       S.si, cap, sb);
    return hipGetLastError();
  }
  for (int c = 0; c < m; ++c) {
    const long long o = (long long)c * sb;
    size_t bytes = S.sort_bytes;
    const hipError_t e = hipcub::DeviceRadixSort::SortPairs(
        offset_bytes(S.sort_tmp, o), bytes, offset_bytes(S.tv, o), offset_bytes(S.sv, o),
        offset_bytes(S.ti, o), offset_bytes(S.si, o), (int)cap, 0, 64, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace

size_t psis_col_stride(long long tail_cap) {
  return (psis_scratch_bytes(tail_cap) + 255) / 256 * 256;
}

// psislw of m columns at once: element (i, c) of lw / out at [c * cs + i * rs]
// (device pointers); column c's scratch at scratch + c * psis_col_stride(Mt).
// Results: k_dev[c], n_tail_dev[c], tail_idx_dev[c * tail_cap + i] (optional).
hipError_t psis_columns(const double* lw, double* out, long long n, int m, long long rs,
                        long long cs, long long Mt, void* scratch, double* k_dev,
                        long long* tail_idx_dev, long long tail_cap, long long* n_tail_dev,
                        hipStream_t s, unsigned* flag_dev, unsigned* flag_host) {
  const long long cap = Mt < 1 ? 1 : Mt;   // the tail holds at most M_t draws
  const long long sb = (long long)psis_col_stride(cap);
  PsisScratch S = carve(scratch, cap);
  const int g = psis_grid(n);
  const size_t sort_lds = (sizeof(unsigned long long) + sizeof(unsigned)) * kTailMax;
  // fast path (see the header): 1 + 2 in two histogram passes; the host reads the
  // per-column flags (one wait) and takes the radix path when any column's
  // candidates exceed one workgroup's sort
  bool fast = flag_dev && flag_host && psis_fast_select_enabled() && cap <= kTailMax && n < (1LL << 31);
  if (fast) {
    hipLaunchKernelGGL(sel_init_kernel, dim3(1, m), dim3(256), 0, s, S.ps, S.hist, n - Mt - 1, sb);
    hipLaunchKernelGGL(sel_hist1_kernel, dim3(g, m), dim3(256), 0, s, lw, n, rs, cs, S.part, S.hist,
                       sb);
    hipLaunchKernelGGL(max_final_kernel, dim3(1, m), dim3(256), 0, s, S.part, g, &S.ps->mx, sb);
    hipLaunchKernelGGL(sel_pick_kernel, dim3(1, m), dim3(256), 0, s, S.hist, S.ps, 1, flag_dev, sb);
    hipLaunchKernelGGL(sel_hist2_kernel, dim3(g, m), dim3(256), 0, s, lw, n, rs, cs, S.ps, S.hist,
                       sb);
    hipLaunchKernelGGL(sel_pick_kernel, dim3(1, m), dim3(256), 0, s, S.hist, S.ps, 2, flag_dev, sb);
    // the flags land in the caller's pinned buffer (the context's, >= m entries)
    unsigned* fl = flag_host;
    hipError_t e = hipMemcpyAsync(fl, flag_dev, sizeof(unsigned) * m, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    for (int c = 0; c < m; ++c) fast = fast && fl[c] == 1u;
  } else {
    hipLaunchKernelGGL(col_max_kernel, dim3(g, m), dim3(256), 0, s, lw, n, rs, cs, S.part, sb);
    hipLaunchKernelGGL(max_final_kernel, dim3(1, m), dim3(256), 0, s, S.part, g, &S.ps->mx, sb);
  }
  if (out)
    hipLaunchKernelGGL(shift_kernel, dim3(g, m), dim3(256), 0, s, lw, out, n, rs, cs, S.ps, sb);
  if (fast) {
    hipLaunchKernelGGL(sel_compact_kernel, dim3(g, m), dim3(256), 0, s, lw, n, rs, cs, S.ps, S.tv,
                       S.ti, sb);
    hipLaunchKernelGGL(sel_sort_kernel, dim3(1, m), dim3(1024), sort_lds, s, S.tv, S.ti, S.ps, S.sv,
                       S.si, n, Mt, log(DBL_MIN), sb);
  } else {
    // 2. radix select of ascending rank n - Mt - 1 (the pick clears the histogram)
    hipLaunchKernelGGL(radix_init_kernel, dim3(1, m), dim3(256), 0, s, S.ps, S.hist, n - Mt - 1, sb);
    for (int pass = 0; pass < 8; ++pass) {
      const int shift = 56 - 8 * pass;
      hipLaunchKernelGGL(radix_hist_kernel, dim3(g, m), dim3(256), 0, s, lw, n, rs, cs, S.ps, shift,
                         S.hist, sb);
      hipLaunchKernelGGL(radix_pick_kernel, dim3(1, m), dim3(256), 0, s, S.hist, shift, S.ps, sb);
    }
    hipLaunchKernelGGL(cutoff_kernel, dim3(1, m), dim3(64), 0, s, S.ps, log(DBL_MIN), sb);
    // 3. stable tail compaction of the shifted values
    const long long chunk = ((n + g - 1) / g + 255) / 256 * 256;
    const int gc = (int)((n + chunk - 1) / chunk);
    // (out null: k and the tails only -- the shift is applied on the fly and the
    // smoothing / renormalisation below, which only feed out, are skipped)
    const int unshifted = out ? 0 : 1;
    const double* sx = out ? out : lw;
    hipLaunchKernelGGL(tail_count_kernel, dim3(gc, m), dim3(256), 0, s, sx, n, rs, cs, chunk, S.ps,
                       S.cnt, sb, unshifted);
    hipLaunchKernelGGL(tail_scan_kernel, dim3(1, m), dim3(64), 0, s, S.cnt, gc, S.ps, sb);
    if (cap > kTailMax)
      hipLaunchKernelGGL(fill_inf_kernel, dim3((unsigned)((cap + 255) / 256), m), dim3(256), 0, s,
                         S.tv, cap, sb);
    hipLaunchKernelGGL(tail_compact_kernel, dim3(gc, m), dim3(256), 0, s, sx, n, rs, cs, chunk,
                       S.ps, S.cnt, cap, S.tv, S.ti, sb, unshifted);
    // 4. sort the tails
    hipError_t e = sort_tail(S, cap, m, sb, s);
    if (e != hipSuccess) return e;
  }
  // 5. GPD fit (skipped on device when n2 <= 4)
  hipLaunchKernelGGL(gpd_prep_kernel, dim3(32, m), dim3(256), 0, s, S.sv, S.ps, S.y, cap, sb);
  const int mmax = 30 + (int)std::sqrt((double)Mt) + 1;
  hipLaunchKernelGGL(gpd_grid_kernel, dim3(mmax, m), dim3(256), 0, s, S.y, S.ps, 0LL, S.bs, S.ks,
                     sb);
  hipLaunchKernelGGL(gpd_final_kernel, dim3(1, m), dim3(256), 0, s, S.y, S.ps, 0LL, S.bs, S.ks,
                     S.Lw, nullptr, nullptr, sb);
  hipLaunchKernelGGL(k_inf_kernel, dim3(1, m), dim3(64), 0, s, S.ps, sb);
  if (!out) {
    const unsigned go = (unsigned)std::max<long long>(1, std::min<long long>(32, (Mt + 255) / 256));
    hipLaunchKernelGGL(psis_out_kernel, dim3(go, m), dim3(256), 0, s, S.ps, S.si, Mt, k_dev,
                       n_tail_dev, tail_idx_dev, tail_cap, sb);
    return hipGetLastError();
  }
  // 6. smoothing
  hipLaunchKernelGGL(smooth_kernel, dim3(32, m), dim3(256), 0, s, out, rs, cs, S.ps, S.si, cap, sb);
  // 7. renormalise: x -= sumlogs(x)
  hipLaunchKernelGGL(col_max_kernel, dim3(g, m), dim3(256), 0, s, out, n, rs, cs, S.part, sb);
  hipLaunchKernelGGL(max_final_kernel, dim3(1, m), dim3(256), 0, s, S.part, g, &S.ps->b, sb);
  hipLaunchKernelGGL(sumexp_kernel, dim3(g, m), dim3(256), 0, s, out, n, rs, cs, &S.ps->b, S.part,
                     sb);
  hipLaunchKernelGGL(lse_final_kernel, dim3(1, m), dim3(256), 0, s, S.part, g, &S.ps->b,
                     &S.ps->lse, sb);
  hipLaunchKernelGGL(sub_kernel, dim3(g, m), dim3(256), 0, s, out, n, rs, cs, &S.ps->lse, sb);
  const unsigned go = (unsigned)std::max<long long>(1, std::min<long long>(32, (Mt + 255) / 256));
  hipLaunchKernelGGL(psis_out_kernel, dim3(go, m), dim3(256), 0, s, S.ps, S.si, Mt, k_dev,
                     n_tail_dev, tail_idx_dev, tail_cap, sb);
  return hipGetLastError();
}

// gpdfitnew on a caller array x[n] (device), any order.  out4 = {k, sigma, m, nkeep}
hipError_t psis_gpdfit(const double* x, long long n, void* scratch, double* out4,
                       double* ks_out, double* w_out, hipStream_t s) {
  PsisScratch S = carve(scratch, n);
  hipLaunchKernelGGL(iota_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n,
                     S.tv, S.ti, S.ps);
  hipError_t e0 = sort_tail(S, n, 1, 0, s);
  if (e0 != hipSuccess) return e0;
  const int m = 30 + (int)std::sqrt((double)n);
  hipLaunchKernelGGL(gpd_grid_kernel, dim3(m), dim3(256), 0, s, S.sv, S.ps, n, S.bs, S.ks, 0LL);
  hipLaunchKernelGGL(gpd_final_kernel, dim3(1), dim3(256), 0, s, S.sv, S.ps, n, S.bs, S.ks, S.Lw,
                     ks_out, w_out, 0LL);
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

// sumlogs of `rows` contiguous rows of n values (row r at x + r n) in one launch
// chain: every kernel takes its row from blockIdx.y; per-row scratch (partials +
// max) sb bytes apart; out[r] dense
__global__ __launch_bounds__(256) void lse_rows_final_kernel(const double* part, int nb,
                                                             const double* mx, double* out,
                                                             long long sb) {
  __shared__ double red[16];
  part = colp(part, sb);
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[b];
  s = bsum(s, red);
  if (threadIdx.x == 0) out[blockIdx.y] = log(s) + *colp(mx, sb);
}

size_t psis_sumlogs_rows_scratch_bytes(long long rows, long long n) {
  return (size_t)rows * (size_t)(psis_grid(n) + 8) * sizeof(double);
}

hipError_t psis_sumlogs_rows(const double* x, long long rows, long long n, void* scratch,
                             double* out, hipStream_t s) {
  const int g = psis_grid(n);
  const long long sb = (long long)(g + 8) * (long long)sizeof(double);
  double* part = static_cast<double*>(scratch);
  double* mx = part + g;
  for (long long r0 = 0; r0 < rows; r0 += 65535) {
    const unsigned R = (unsigned)std::min<long long>(65535, rows - r0);
    const double* xr = x + r0 * n;
    hipLaunchKernelGGL(col_max_kernel, dim3(g, R), dim3(256), 0, s, xr, n, 1LL, n, part, sb);
    hipLaunchKernelGGL(max_final_kernel, dim3(1, R), dim3(256), 0, s, part, g, mx, sb);
    hipLaunchKernelGGL(sumexp_kernel, dim3(g, R), dim3(256), 0, s, xr, n, 1LL, n, mx, part, sb);
    hipLaunchKernelGGL(lse_rows_final_kernel, dim3(1, R), dim3(256), 0, s, part, g, mx, out + r0,
                       sb);
  }
  return hipGetLastError();
}

hipError_t psis_sumlogs(const double* x, long long n, void* scratch, double* out, hipStream_t s) {
  PsisScratch S = carve(scratch, 0);
  const int g = psis_grid(n);
  hipLaunchKernelGGL(col_max_kernel, dim3(g), dim3(256), 0, s, x, n, 1LL, 0LL, S.part, 0LL);
  hipLaunchKernelGGL(max_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b, 0LL);
  hipLaunchKernelGGL(sumexp_kernel, dim3(g), dim3(256), 0, s, x, n, 1LL, 0LL, &S.ps->b, S.part,
                     0LL);
  hipLaunchKernelGGL(lse_final_kernel, dim3(1), dim3(256), 0, s, S.part, g, &S.ps->b, out, 0LL);
  return hipGetLastError();
}

}  // namespace vbk

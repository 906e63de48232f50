// vb_gemm.hpp — fp64 GEMM on CDNA4 matrix cores (v_mfma_f64_16x16x4_f64) with
// the epilogues the full-rank path fuses (row divide, column bias, beta C).
//
// C[M][N] = alpha * op(A) diag(kscale) op(B) [/ row_div[i]] [+ col_bias[j]] [+ diag I] + beta C
// (row-major, leading dimensions lda/ldb/ldc; op = transpose when ta / tb).
//
// Block tile 32 x 32 computed by 8 waves: 4 output quadrants of 16 x 16 x 2 halves
// of every k tile (intra-block split-K, reduced through LDS at the end), each
// wave running 4 independent MFMA accumulator chains.  K is staged KT (32) at a
// time through double-buffered LDS with the next tile's global loads in flight
// while the current one feeds the MFMAs (one barrier per tile).
// LDS layout per operand follows its contiguous global dimension so both the
// coalesced store and the fragment read are conflict-free at the 2-pass minimum:
//   contiguous in k  -> [row][k]  (stride 34 doubles)
//   contiguous in row -> [k][row] (stride 48 doubles)
// MFMA operand maps (cdna_hip_programming.md): A[l&15][k=l>>4], B[k=l>>4][l&15];
// C row = (l>>4) + 4 r, col = l&15.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

namespace vbk {

// Touch every 64-byte line of a kernel's by-value argument struct at once.
// The fields are read later behind data-dependent scalar branches, and each
// line's first read is a scalar-cache miss (kernel arguments live in HBM) that
// the wave waits on; one overlapped round of misses replaces several serial
// ones (about 0.5 us each; measured on the fp64 GEMM, profiles/r03/cfg4).
template <class T>
__device__ __forceinline__ void kernarg_warm(const T& a) {
  constexpr int W = (int)(sizeof(T) / 4), NL = (W + 15) / 16 + 1;
  const int* p = reinterpret_cast<const int*>(&a);
  int x = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) x ^= p[16 * i < W ? 16 * i : W - 1];
  asm volatile("" ::"s"(x));
}

struct GemmOp {
  bool ta, tb;
  int M, N, K;
  const double* A;
  long long lda;
  const double* B;
  long long ldb;
  double* C;
  long long ldc;
  double alpha, beta;
  const double* kscale;    // [K] or null
  const double* row_div;   // [M] or null
  const double* col_bias;  // [N] or null
  double diag;             // added to C[i][i] (after the bias)
  // optional second product accumulated into the same C (same shapes, leading
  // dimensions and transposes): C = alpha op(A) op(B) + alpha2 op(A2) op(B2) ...
  const double* A2;
  const double* B2;
  double alpha2;
  // optional: per-wave partial sums of (C_ij - sq_shift [i == j])^2 over the
  // written outputs, 4 per block at sq_part[4 (by gridDim.x + bx) + wave]
  double* sq_part;
  double sq_shift;
  // ---- device-resident scalars and control (the sync-free full-rank step) ----
  const double* alpha_dev;     // alpha (and alpha2) *= *alpha_dev
  const double* sq_shift_dev;  // overrides sq_shift
  // skip: when *skip_flag was set by an EARLIER launch the block copies copy_src
  // into C (if given) or returns.  Convergence test run first by every block, in
  // the same fixed order: s = conv_scale * sum(conv_part[0, conv_n)); if s <=
  // conv_tol2 * (*conv_ref or 1) the block sets *skip_flag = skip_tag and writes
  // conv_iter to *conv_iter_out, then skips.  A launch that writes the flag
  // carries a tag (> 0) distinct from every other launch that writes the same
  // flag in one step: a block that finds its OWN launch's tag (a peer block got
  // there first) ignores it and runs the test itself -- every block sums the same
  // partials in the same order, so all decide alike, and no block depends on the
  // order in which peers' stores to the flag and to conv_iter_out become visible.
  int* skip_flag;
  int skip_tag;
  const double* copy_src;
  const double* conv_part;
  int conv_n;
  const double* conv_scale_dev;
  const double* conv_ref_dev;
  double conv_tol2;
  // stall: also converged when s <= conv_stall_tol2 * ref and the previous
  // iterate's sum s_prev (conv_prev_part, same count, same scale rule with
  // conv_prev_scale_dev) satisfies s >= s_prev / 16 (rounding floor reached)
  const double* conv_prev_part;
  const double* conv_prev_scale_dev;
  double conv_stall_tol2;
  int* conv_iter_out;
  int conv_iter;
  // finish-after-update (Newton-Schulz): when the test sum s <= conv_fin_tol2 *
  // ref (and the skip test failed) the block computes its tile as usual and sets
  // *fin_flag = 1 and *conv_iter_out = conv_iter + 1: the next iterate is final.
  // Later launches name fin_flag as skip_flag2: they skip (setting *skip_flag).
  int* fin_flag;
  double conv_fin_tol2;
  const int* skip_flag2;
  // copy_src applies only in the first skipped launch after convergence
  // (copy_if_iter = that launch's iteration; -1: always): the launch whose own
  // test converged (conv_iter == copy_if_iter), or a launch skipped by an earlier
  // one with *conv_iter_out == copy_if_iter
  int copy_if_iter;
  // optional: per-wave partial sums of dot_with_ij * C_ij (before beta), 4 per block
  const double* dot_with;
  double* dot_part;
  // Newton-Schulz iteration 0 (A = B = Sigma): C = ns0[0] Sigma^2 + ns0[1] Sigma and
  // ns0_z = ns0[2] (3 I - ns0[3] Sigma), written for the same tile
  const double* ns0;
  double* ns0_z;
  // optional per-row partials of the written tile, 2 per 32-column tile (one per
  // 16-column quadrant) at rp_part[(2 bx + quadrant column) M + row]:
  //   rp_x: sum_j C_ij rp_x[j]  (a matrix-vector product: a power step on C)
  //   rp_w: sum_j C_ij rp_w[i][j] (leading dimension ldc; a row-wise dot product)
  const double* rp_x;
  const double* rp_w;
  double* rp_part;
  // optional: per-wave partial sums of qf_x_i C_ij qf_x_j (a quadratic form of
  // the written tile), 4 per block at qf_part[4 (by gridDim.x + bx) + wave]
  const double* qf_x;
  double* qf_part;
  // symmetric result (M == N, the caller's guarantee that C is symmetric in exact
  // arithmetic): only the tiles (bi <= bj) of the upper triangle are computed, one
  // block each, and every off-diagonal tile is also stored transposed into
  // (bj, bi); partial sums (sq_part, qf_part, dot_part) weight off-diagonal tiles
  // twice and are indexed by the triangular block index (4 nt (nt + 1) / 2 in all)
  int sym;
  // set by gemm_group: M, N multiples of 32, K of KTG, 16-byte aligned operand rows, no
  // kscale / dual product -> the LDS-DMA main loop
  int glds;
  // stream-K (the grouped Newton-Schulz Y|Z product, gemm_group): when set on both ops
  // of a symmetric pair whose tiles slightly outnumber the CUs, the k stages of all
  // tiles are dealt evenly over one block per CU; a tile split between two blocks is
  // finished by the block holding its first stages, which adds the partial tile the
  // other block left in sk_part[tile] (flagged sk_flag[tile] = sk_epoch, a value
  // distinct per launch).  Scratch: 1024 doubles and one int per tile of the pair.
  double* sk_part;
  int* sk_flag;
  int sk_epoch;
};

// Up to two independent GEMMs of equal shape / transposes in one launch
// (blockIdx.z selects the problem).
struct GemmGroup {
  GemmOp op[2];
};

// Epilogue / control features of a GemmOp as compile-time bits.  A kernel
// instantiated for an exact feature set (gemm_group picks one of the sets the
// full-rank step uses) carries only that code: each launch runs its entry and
// epilogue from a cold instruction cache (the store phase takes ~1 us the first
// time and 0.3 us when run again, profiles/r04), so the once-per-launch code is
// kept short and straight.  kEpiAll: every feature tested at run time.
enum : int {
  kEpiRowDiv = 1, kEpiColBias = 2, kEpiDiag = 4, kEpiNs0 = 8, kEpiDot = 16, kEpiRpX = 32,
  kEpiQf = 64, kEpiRpW = 128, kEpiBeta = 256, kEpiSq = 512, kEpiAlphaDev = 1024,
  kEpiShiftDev = 2048, kEpiSym = 4096, kEpiSkip = 8192, kEpiAll = 16383
};

namespace gemm_detail {

using d4 = double __attribute__((ext_vector_type(4)));
constexpr int BT = 32;   // block tile (rows and columns)
#ifndef VB_GEMM_KT
#define VB_GEMM_KT 32
#endif
constexpr int KT = VB_GEMM_KT;  // k tile
constexpr int SR = KT + 2;      // [row][k] stride: 2 SR = 4 (mod 64 banks), so a 32-lane
                                // pass of fragment reads (16 rows x 2 k) hits 64 distinct banks
constexpr int SK = BT + 16;     // [k][row] stride
constexpr int BUF = (BT * SR > KT * SK) ? BT * SR : KT * SK;  // doubles per operand buffer
#ifndef VB_GEMM_KSPLIT
#define VB_GEMM_KSPLIT 2
#endif
constexpr int KS_ = VB_GEMM_KSPLIT;                            // k parts of each tile
constexpr int NTH = 256 * KS_;                                 // 4 quadrants x KS_ waves
constexpr int PER = BT * KT / NTH;                             // elements per thread per tile

// One operand tile (BT rows x KT k) of a row-major matrix X with leading
// dimension ld; KCONTIG: X is [row][k] in memory (k contiguous), else [k][row].
// Loads are branch-free: an element outside the matrix reads element 0 and
// is zeroed (and k-scaled) only at store time, so no use of a loaded value and
// no per-lane branch sits between a tile's loads and its store to LDS.  The
// compiler then waits (s_waitcnt vmcnt) for exactly the tile being stored while
// the next tile's loads stay in flight; guarded loads had made it wait for every
// outstanding load (vmcnt(0)) on each k tile.
template <bool KCONTIG, bool KS>
struct Tile {
  double v[PER];
  double ks[KS ? PER : 1];
  bool ok[PER];
  // loop-invariant per-thread layout: element offsets from the tile base (a
  // uniform pointer), row in range, k within the tile
  unsigned off[PER], offr[PER];   // offr: 0 when the row is out of range
  int kk[PER];
  bool rok[PER];
  __device__ __forceinline__ void init(long long ld, int r0, int R, int t) {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = t + NTH * e;
      const int r = KCONTIG ? idx / KT : idx % BT;
      const int k = KCONTIG ? idx % KT : idx / BT;
      off[e] = KCONTIG ? (unsigned)(r * ld + k) : (unsigned)(k * ld + r);
      rok[e] = r0 + r < R;
      offr[e] = rok[e] ? off[e] : 0u;
      kk[e] = k;
    }
  }
  __device__ __forceinline__ void load(const double* X, long long ld, int r0, int k0, int K,
                                       const double* kscale) {
    const double* base = X + (KCONTIG ? (long long)r0 * ld + k0 : (long long)k0 * ld + r0);
    const int kl = K - k0;
    if (kl >= KT) {   // whole k tile inside K (uniform): invariant offsets, no per-load math
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        v[e] = base[offr[e]];
        if constexpr (KS) ks[e] = kscale[k0 + kk[e]];
        ok[e] = rok[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const bool in = rok[e] && kk[e] < kl;
        v[e] = base[in ? off[e] : 0u];
        if constexpr (KS) ks[e] = kscale[in ? k0 + kk[e] : 0];
        ok[e] = in;
      }
    }
  }
  __device__ __forceinline__ void store(double* s, int t) const {
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int idx = t + NTH * e;
      const int r = KCONTIG ? idx / KT : idx % BT;
      const int k = KCONTIG ? idx % KT : idx / BT;
      const double x = KS ? v[e] * ks[KS ? e : 0] : v[e];
      s[KCONTIG ? r * SR + k : k * SK + r] = ok[e] ? x : 0.0;
    }
  }
};

template <bool KCONTIG>
__device__ __forceinline__ double frag(const double* s, int r, int k) {
  return KCONTIG ? s[r * SR + k] : s[k * SK + r];
}

// Block-uniform skip decision (see GemmOp::skip_flag): 0 = compute the tile;
// 1 = skipped (converged in an earlier launch); 2 = skipped (this launch's own
// convergence test).  Every block sums the partials in the same order, so all
// blocks decide alike.
template <int EPI = kEpiAll>
__device__ __forceinline__ int gemm_skip(const GemmOp& g, double* red) {
  if constexpr (!(EPI & kEpiSkip)) return 0;
  if (!g.skip_flag) return 0;
  __shared__ int s_skip;
  const int t = threadIdx.x;
  if (g.conv_part) {
    double a = 0.0, b = 0.0;
    for (int i = t; i < g.conv_n; i += NTH) {
      a += g.conv_part[i];
      if (g.conv_prev_part) b += g.conv_prev_part[i];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a += __shfl_xor(a, off, 64);
      b += __shfl_xor(b, off, 64);
    }
    if ((t & 63) == 0) {
      red[t >> 6] = a;
      red[NTH / 64 + (t >> 6)] = b;
    }
  }
  __syncthreads();
  if (t == 0) {
    const int tag = g.skip_tag > 0 ? g.skip_tag : 1;
    const int f = __hip_atomic_load(g.skip_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a flag holding this launch's own tag was set by a peer block: ignore it
    int sk = (f != 0 && !(g.skip_tag > 0 && f == g.skip_tag)) ? 1 : 0;
    if (!sk && g.skip_flag2 && *g.skip_flag2 != 0) {
      sk = 1;
      __hip_atomic_store(g.skip_flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!sk && g.conv_part) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < NTH / 64; ++k) {
        a += red[k];
        b += red[NTH / 64 + k];
      }
      if (g.conv_scale_dev) a *= *g.conv_scale_dev;
      if (g.conv_prev_scale_dev) b *= *g.conv_prev_scale_dev;
      const double ref = g.conv_ref_dev ? *g.conv_ref_dev : 1.0;
      const bool stall = g.conv_prev_part && a <= g.conv_stall_tol2 * ref && a * 16.0 >= b;
      if (a <= g.conv_tol2 * ref || stall) {
        sk = 2;
        if (g.conv_iter_out) *g.conv_iter_out = g.conv_iter;
        __hip_atomic_store(g.skip_flag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (g.fin_flag && a <= g.conv_fin_tol2 * ref) {
        *g.fin_flag = 1;
        if (g.conv_iter_out) *g.conv_iter_out = g.conv_iter + 1;
      }
    }
    s_skip = sk;
  }
  __syncthreads();
  return s_skip;
}

// ---- LDS-DMA main loop (M, N, K multiples of KTG; no kscale / dual product) ----
// Operand tiles go global -> LDS directly (global_load_lds_dwordx4: no VGPR
// staging, so no register of an in-flight load is ever reused and the loop
// keeps GS - 1 tiles in flight across its barriers).  A stage holds KTG (64) k
// of both operands: a tile is "rows" of the operand's contiguous global
// dimension (RL doubles each: KTG for k-contiguous operands, BT for
// row-contiguous ones); one wave instruction moves 1 KB, each lane 16 B (a pair
// of doubles), and each wave issues KTG / 32 instructions per operand and
// stage.  The LDS destination of a lane is fixed (instruction base + 16 lane),
// so the bank swizzle is applied to the GLOBAL address: LDS slot s of row r
// holds element s ^ sw(r) (pairs stay pairs: sw even).
//   rows = m / n, k contiguous (A, or B^T):  sw(r) = 2 (r & 15)  -- a fragment
//     read (16 rows x 2 k per 32 lanes) then covers 64 distinct banks (row
//     stride KTG doubles = 0 mod 64 banks);
//   rows = k, m / n contiguous (A^T, or B): sw(r) = 16 (r & 1)   -- rows k, k+1
//     land in opposite bank halves.
// Within a stage, wave (quadrant q, k part h) consumes k = 32 u + 16 h + 4 s + kq
// (sub-tile u, step s) into accumulator chain s: the k order of every chain is
// that of the register-staged loop (KT = 32), so both loops give the same bits.
// (Sweep over k depth x stages, profiles/r03/gemm_glds_sweep.log: 64 x 2 is the
// fastest, 10.5 us per cold 512^3 product against 11.2 for 32 x 4.)
#ifndef VB_GEMM_GS
#define VB_GEMM_GS 2
#endif
#ifndef VB_GEMM_KTG
#define VB_GEMM_KTG 64
#endif
constexpr int GS = VB_GEMM_GS;   // LDS stages (tiles it+1 .. it+GS-1 in flight)
constexpr int KTG = VB_GEMM_KTG; // k per stage
static_assert(KTG % 32 == 0 && KT == 32 && KS_ == 2, "LDS-DMA loop: 32-deep sub-tiles, 2 k parts");
constexpr int NSUB = KTG / 32;   // 32-deep sub-tiles per stage
constexpr int TD = BT * KTG;     // doubles per operand tile
constexpr int SMEM = (4 * BUF > 2 * GS * TD) ? 4 * BUF : 2 * GS * TD;  // doubles of LDS per block
static_assert(SMEM * 8 <= 65536, "static LDS of one block");
template <bool KROWS>
__device__ __forceinline__ int swz(int r) { return KROWS ? 2 * (r & 15) : 16 * (r & 1); }
template <bool KROWS>
constexpr int row_len() { return KROWS ? KTG : BT; }

// Global element offset (from the tile origin) that lane `lane` of wave `w`
// loads for its 16-byte LDS slot in instruction j; ld = leading dimension.
template <bool KROWS>
__device__ __forceinline__ long long glds_src(int j, int w, int lane, long long ld) {
  constexpr int RL = row_len<KROWS>();
  const int o = (j * 8 + w) * 128 + 2 * lane;   // LDS double offset within the tile
  const int r = o / RL, s = o % RL;
  return (long long)r * ld + (s ^ swz<KROWS>(r));
}

// LDS offset (doubles) of fragment element (row r, column c) of a tile laid
// out with `rows` = r.
template <bool KROWS>
__device__ __forceinline__ int glds_at(int r, int c) {
  return r * row_len<KROWS>() + (c ^ swz<KROWS>(r));
}

// each wave has 2 NSUB LDS-DMA instructions per tile (A, B) in flight
__device__ __forceinline__ void vm_wait_tiles(int pending) {
  static_assert(GS <= 4 && 2 * NSUB * 3 <= 63, "vmcnt range");
  if (pending >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * NSUB) : "memory");
  else if (pending == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NSUB) : "memory");
  else if (pending == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NSUB) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#ifdef VB_GEMM_PROF
// phase timestamps (s_memrealtime, 100 MHz) of thread 0 of every block of the
// last launch: [0] entry, [1] after the skip test, [2] main loop start,
// [3..10] after each of the first 8 k stages' barriers, [14] main loop end, [16]
// accumulators summed (MFMA results in registers), [11] k parts reduced, [17]
// epilogue operands read (alpha, partners' sums), [12] tile stored, [13] partial
// sums stored, [15] epilogue end
__device__ unsigned long long g_gemm_ts[1024][24];
#define VB_GEMM_TS(k)                                                                \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x + blockIdx.y * gridDim.x < 1024)              \
      g_gemm_ts[blockIdx.x + blockIdx.y * gridDim.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define VB_GEMM_TS(k) do {} while (0)
#endif

// KSC: the A fragments are scaled by a per-k factor read from LDS (ks, K
// doubles), after the fragment reads: the same product a * ks that the
// register-staged loop forms at its LDS store, so the bits are the same.  mid()
// runs after the first stages are issued (a hook's loads then overlap them).
template <bool TA, bool TB, bool KSC, class Mid>
__device__ __forceinline__ void mainloop_glds(const GemmOp& g, int i0, int j0, double* lds,
                                              d4 (&acc)[4], const double* ks, Mid&& mid,
                                              int st0 = 0, int nst = -1) {
  // A rows: m when not transposed (k contiguous), k when transposed.
  // B rows: n when transposed (k contiguous), k otherwise.
  constexpr bool AK = !TA, BK = TB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = w & 3, h = w >> 2;
  const int wm = q >> 1, wn = q & 1;
  double* sA = lds;                 // [GS][TD]
  double* sB = lds + GS * TD;       // [GS][TD]
  // (stream-K: the k stages [st0, st0 + nst) only)
  const int nt = nst < 0 ? g.K / KTG : nst;
  // per-lane global sources: tile origin + fixed offsets; the origin moves by KTG
  // along k each tile (k is the row index of the "rows = k" layouts)
  const long long kb0 = (long long)st0 * KTG;
  const double* a0 = g.A + (AK ? (long long)i0 * g.lda + kb0 : (long long)i0 + kb0 * g.lda);
  const double* b0 = g.B + (BK ? (long long)j0 * g.ldb + kb0 : (long long)j0 + kb0 * g.ldb);
  long long aoff[NSUB], boff[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j) {
    aoff[j] = glds_src<AK>(j, w, lane, g.lda);
    boff[j] = glds_src<BK>(j, w, lane, g.ldb);
  }
  const long long astep = AK ? KTG : (long long)KTG * g.lda;
  const long long bstep = BK ? KTG : (long long)KTG * g.ldb;
  auto issue = [&](int it) {
    const int st = it % GS;
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      __builtin_amdgcn_global_load_lds((const void*)(a0 + it * astep + aoff[j]),
                                       (void*)(sA + st * TD + 128 * (j * 8 + w)), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(b0 + it * bstep + boff[j]),
                                       (void*)(sB + st * TD + 128 * (j * 8 + w)), 16, 0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < GS - 1; ++s)
    if (s < nt) issue(s);
  mid();
  // fragment offsets within a stage for this wave's 4 NSUB k4-steps (sub-tile u,
  // step s: k = 32 u + 16 h + 4 s + kq)
  const int ra = wm * 16 + (lane & 15), cb = wn * 16 + (lane & 15), kq = lane >> 4;
  constexpr int NST = 4 * NSUB;
  typedef __attribute__((address_space(3))) double lds_f64;
  const unsigned la = (unsigned)(uintptr_t)((lds_f64*)sA), lb = (unsigned)(uintptr_t)((lds_f64*)sB);
  unsigned xa[NST], xb[NST], xk[KSC ? NST : 1];
  const unsigned lk = KSC ? (unsigned)(uintptr_t)((const lds_f64*)ks) : 0u;
#pragma unroll
  for (int f = 0; f < NST; ++f) {
    const int kk = 32 * (f >> 2) + 16 * h + 4 * (f & 3) + kq;
    xa[f] = la + 8u * (unsigned)(AK ? glds_at<true>(ra, kk) : glds_at<false>(kk, ra));
    xb[f] = lb + 8u * (unsigned)(BK ? glds_at<true>(cb, kk) : glds_at<false>(kk, cb));
    if constexpr (KSC) xk[f] = lk + 8u * (unsigned)kk;
  }
  VB_GEMM_TS(2);
  for (int it = 0; it < nt; ++it) {
    const int last_issued = it + GS - 2 < nt - 1 ? it + GS - 2 : nt - 1;
    vm_wait_tiles(last_issued - it);
    __builtin_amdgcn_s_barrier();            // tile it is in LDS; stage (it - 1) % GS is free
    if (it < 8) VB_GEMM_TS(3 + it);
#ifndef VB_GEMM_NOLOAD
    if (it + GS - 1 < nt) issue(it + GS - 1);
#endif
    // fragment reads as inline asm: the compiler would otherwise guard every
    // ds_read behind vmcnt(0) (it cannot tell which LDS-DMA tile a read
    // aliases), draining the tiles in flight; the waits below are explicit.
    // Four steps' reads (8) stay in flight: step f + 4 is issued after step f's
    // MFMA, into its own registers (lgkmcnt counts LDS reads in order)
    const unsigned so = (unsigned)((it % GS) * TD * 8);
    const unsigned ko = (unsigned)(it * KTG * 8);
    double fa[NST], fb[NST], fk[KSC ? NST : 1];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      asm volatile("ds_read_b64 %0, %1" : "=v"(fa[f]) : "v"(xa[f] + so));
      asm volatile("ds_read_b64 %0, %1" : "=v"(fb[f]) : "v"(xb[f] + so));
      if constexpr (KSC) asm volatile("ds_read_b64 %0, %1" : "=v"(fk[f]) : "v"(xk[f] + ko));
    }
#pragma unroll
    for (int f = 0; f < NST; ++f) {
      const int ahead = (NST - 1 - f) < 3 ? (NST - 1 - f) : 3;   // steps issued after f
      if constexpr (KSC) {   // three reads per step
        if (ahead == 3) asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(fa[f]), "+v"(fb[f]), "+v"(fk[f]));
        else if (ahead == 2) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(fa[f]), "+v"(fb[f]), "+v"(fk[f]));
        else if (ahead == 1) asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(fa[f]), "+v"(fb[f]), "+v"(fk[f]));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[f]), "+v"(fb[f]), "+v"(fk[f]));
        fa[f] *= fk[f];
      } else {
        if (ahead == 3) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(fa[f]), "+v"(fb[f]));
        else if (ahead == 2) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(fa[f]), "+v"(fb[f]));
        else if (ahead == 1) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(fa[f]), "+v"(fb[f]));
        else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[f]), "+v"(fb[f]));
      }
#ifdef VB_GEMM_NOMFMA
      acc[f & 3][0] += fa[f] * fb[f];
#else
      acc[f & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[f], fb[f], acc[f & 3], 0, 0, 0);
#endif
// (rejected: issuing the next stage's LDS-DMA pieces one per MFMA step instead
      // of after the barrier -- 9.66 / 9.78 vs 9.67 / 9.51 us per cold 512^3
      // product, scripts/ubench/gemm_chain.cpp, profiles/r05/dma_interleave_rejected.log)
      if (f + 4 < NST) {
        asm volatile("ds_read_b64 %0, %1" : "=v"(fa[f + 4]) : "v"(xa[f + 4] + so));
        asm volatile("ds_read_b64 %0, %1" : "=v"(fb[f + 4]) : "v"(xb[f + 4] + so));
        if constexpr (KSC)
          asm volatile("ds_read_b64 %0, %1" : "=v"(fk[f + 4]) : "v"(xk[f + 4] + ko));
      }
    }
  }
  __syncthreads();
  VB_GEMM_TS(14);
}

// One BT x BT output tile (bx, by) of g (the whole block, NTH threads).  slot =
// the block's partial-sum index.  sA / sB: the block's LDS operand buffers.
// Ends with a barrier, so a caller may run further tiles on the same buffers.
// Upper-triangle tile (bi <= bj) of triangular block index b (row-major over bi).
__device__ __forceinline__ void tri_tile(int b, int nt, int& bi, int& bj) {
  int i = 0;
  while (b >= nt - i) {
    b -= nt - i;
    ++i;
  }
  bi = i;
  bj = i + b;
}

// A GEMM kernel may carry a hook (gemm_f64_hook_kernel): pre() runs before the
// main loop (e.g. issues loads whose latency then hides under it), post(lds)
// after it; a non-null return of post is a block-local Newton-Schulz iteration-0
// coefficient set used in place of GemmOp::ns0 (a schedule the block computed).
// A stream-K part of a tile (gemm_f64_sk_kernel): k stages [st0, st0 + nst); mode 0 the
// whole tile (nst < 0: all stages), 1 a later part whose partial tile goes to part and
// flag, 2 the first part, which waits for the flag, adds the partial and finishes.
struct SkPart {
  int mode = 0, st0 = 0, nst = -1;
  double* part = nullptr;
  int* flag = nullptr;
  int epoch = 0;
};

struct NoHook {
  static constexpr bool kKScale = false;   // pre() leaves K scales of A in LDS (kscale())
  static constexpr int kLds = 1;           // doubles of LDS scratch the hook uses
  static constexpr int kEpi = kEpiAll;     // epilogue feature set of the hooked product
  __device__ __forceinline__ void pre() {}
  __device__ __forceinline__ const double* post() { return nullptr; }
  __device__ __forceinline__ const double* kscale() const { return nullptr; }
};

template <bool TA, bool TB, bool KS, bool DUAL, int EPI = kEpiAll, class Hook = NoHook>
__device__ __forceinline__ void gemm_tile(const GemmOp& g, int bx, int by, int slot,
                                          double (*sA)[BUF], double (*sB)[BUF], double* lds,
                                          Hook&& hook = Hook{}, const SkPart& sk = SkPart{}) {
  // feature f is compiled in when its bit is set; an exact set also drops the
  // run-time null test of its fields
  constexpr bool kExact = EPI != kEpiAll;
  auto has = [&](int f, bool rt) __attribute__((always_inline)) {
    return (EPI & f) && (kExact || rt);
  };
  using H = std::decay_t<Hook>;
  constexpr bool kHook = !std::is_same_v<H, NoHook>;
  // A is k-contiguous when not transposed; B is k-contiguous when transposed.
  constexpr bool AK = !TA, BK = TB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = w & 3, h = w >> 2;           // output quadrant, k part of each tile
  const int wm = q >> 1, wn = q & 1;
  const int i0 = by * BT, j0 = bx * BT;
  const int kq = lane >> 4;
  // four independent accumulator chains (interleaved k4 steps): one dependent
  // f64 MFMA chain per wave is latency-bound on gfx950
  d4 acc[4], acc2[DUAL ? 4 : 1];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < (DUAL ? 4 : 1); ++c) acc2[c] = d4{0.0, 0.0, 0.0, 0.0};
#ifdef VB_GEMM_EXP_CTOUCH
  {   // experiment: touch this thread's output rows before the main loop (TLB / L2)
    const int col_ = j0 + wn * 16 + (lane & 15), row_ = i0 + wm * 16 + kq;
    if (h == 0 && row_ < g.M && col_ < g.N) {
      double t_;
      asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(t_) : "v"(g.C + (long long)row_ * g.ldc + col_));
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(t_));
    }
  }
#endif
  bool done = false;
  if constexpr (!KS && !DUAL) {
    if (g.glds) {   // aligned shapes: LDS-DMA main loop (same k order, same bits)
      mainloop_glds<TA, TB, H::kKScale>(g, i0, j0, lds, acc, hook.kscale(), [&]() {
        if constexpr (kHook) hook.pre();
      }, sk.st0, sk.nst);
      done = true;
    }
  }
  // (a hook that scales K runs on the LDS-DMA loop only: gemm_hook checks)
  if constexpr (kHook && !H::kKScale) {
    if (!done) hook.pre();
  }
  if (!done) {
  const int nt1 = (g.K + KT - 1) / KT;
  const int nt = DUAL ? 2 * nt1 : nt1;   // the second product's tiles follow the first's
  // tile `it` of the virtual k range: operands and k offset
  auto src_a = [&](int it) { return (DUAL && it >= nt1) ? g.A2 : g.A; };
  auto src_b = [&](int it) { return (DUAL && it >= nt1) ? g.B2 : g.B; };
  auto koff = [&](int it) { return (DUAL && it >= nt1 ? it - nt1 : it) * KT; };
  // prefetches past the last tile re-read the last one (unconditional loads keep
  // the instruction stream straight for the waitcnt placement; the copy is unused)
  auto cl = [&](int it) { return it < nt ? it : nt - 1; };
  // two register stages: tile it+2 is loaded while tile it feeds the MFMAs
  // and tile it+1 (loaded one iteration earlier) moves to LDS
  Tile<AK, KS> ta0, ta1;
  Tile<BK, false> tb0, tb1;
  ta0.init(g.lda, i0, g.M, t);
  ta1.init(g.lda, i0, g.M, t);
  tb0.init(g.ldb, j0, g.N, t);
  tb1.init(g.ldb, j0, g.N, t);
  ta0.load(src_a(0), g.lda, i0, koff(0), g.K, g.kscale);
  tb0.load(src_b(0), g.ldb, j0, koff(0), g.K, nullptr);
  ta1.load(src_a(cl(1)), g.lda, i0, koff(cl(1)), g.K, g.kscale);
  tb1.load(src_b(cl(1)), g.ldb, j0, koff(cl(1)), g.K, nullptr);
  ta0.store(sA[0], t);
  tb0.store(sB[0], t);
  __syncthreads();
  const int ra = wm * 16 + (lane & 15), cb = wn * 16 + (lane & 15);
  const int kb = h * (KT / KS_);
  auto mma = [&](const double* a_s, const double* b_s, int it) {
    if (DUAL && it >= nt1) {
#pragma unroll
      for (int s = 0; s < KT / (4 * KS_); ++s) {
        const int kk = kb + 4 * s;
        const double a = frag<AK>(a_s, ra, kk + kq);
        const double b = frag<BK>(b_s, cb, kk + kq);
        acc2[s & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc2[s & 3], 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < KT / (4 * KS_); ++s) {
      const int kk = kb + 4 * s;
      const double a = frag<AK>(a_s, ra, kk + kq);
      const double b = frag<BK>(b_s, cb, kk + kq);
      acc[s & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s & 3], 0, 0, 0);
    }
  };
  for (int it = 0; it < nt; it += 2) {
    ta0.load(src_a(cl(it + 2)), g.lda, i0, koff(cl(it + 2)), g.K, g.kscale);
    tb0.load(src_b(cl(it + 2)), g.ldb, j0, koff(cl(it + 2)), g.K, nullptr);
    mma(sA[0], sB[0], it);
    if (it + 1 < nt) {
      ta1.store(sA[1], t);
      tb1.store(sB[1], t);
    }
    __syncthreads();
    if (it + 1 >= nt) break;
    ta1.load(src_a(cl(it + 3)), g.lda, i0, koff(cl(it + 3)), g.K, g.kscale);
    tb1.load(src_b(cl(it + 3)), g.ldb, j0, koff(cl(it + 3)), g.K, nullptr);
    mma(sA[1], sB[1], it + 1);
    if (it + 2 < nt) {
      ta0.store(sA[0], t);
      tb0.store(sB[0], t);
    }
    __syncthreads();
  }
  }
  d4 r4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
#ifdef VB_GEMM_PROF
  asm volatile("" : "+v"(r4));
#endif
  VB_GEMM_TS(16);
  if constexpr (DUAL) {
    const d4 r2 = (acc2[0] + acc2[1]) + (acc2[2] + acc2[3]);
    // combine here so the epilogue's alpha applies to both: alpha r + alpha2 r2
    r4 = r4 + (g.alpha2 / g.alpha) * r2;
  }
  // hook: after the main loop
  // (the epilogue's device scalars are read after the main loop: loaded before
  // it, they stay live across it and push the kernel past the 128 VGPRs that two
  // 512-thread blocks per CU allow -- the grouped Y|Z launch then runs in two
  // rounds, 15.8 -> 19.0 us)
  const double* ns0 = g.ns0;
  if constexpr (kHook) {
    const double* h = hook.post();
    if (h) ns0 = h;
  }
  // k parts 1.. hand their partial tiles to part 0 through LDS (fixed order)
  double* red = sA[0];
  if (h >= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((h - 1) * 16 + q * 4 + r) * 64 + lane] = r4[r];
  }
  __syncthreads();
  VB_GEMM_TS(11);
  if (sk.mode == 2 && t == 0) {
    // the tile's later stages: wait (bounded) for the partner block's partial tile
    int it = 0;
    while (__hip_atomic_load(sk.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != sk.epoch &&
           it < (1 << 22)) {
      __builtin_amdgcn_s_sleep(1);
      ++it;
    }
  }
  if (sk.mode == 2) __syncthreads();
  if (h == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double p = red[(q * 4 + r) * 64 + lane];
#pragma unroll
      for (int hh = 2; hh < KS_; ++hh) p += red[((hh - 1) * 16 + q * 4 + r) * 64 + lane];
      r4[r] += p;
    }
    if (sk.mode == 1) {
      // a later part: the partial tile (device-coherent stores) for the first part's
      // block; the flag follows once every thread's stores have completed (below)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __hip_atomic_store(sk.part + (q * 4 + r) * 64 + lane, r4[r], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (sk.mode == 2) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        r4[r] += __hip_atomic_load(sk.part + (q * 4 + r) * 64 + lane, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (sk.mode == 1) {
    __syncthreads();
    if (t == 0) __hip_atomic_store(sk.flag, sk.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (h == 0) {
    const int col = j0 + wn * 16 + (lane & 15);
    double sq = 0.0, dt = 0.0, qf = 0.0, rp[4] = {0.0, 0.0, 0.0, 0.0};
    const bool mirror = has(kEpiSym, g.sym) && bx != by;   // also store the tile transposed
    const bool is_ns0 = has(kEpiNs0, ns0 != nullptr);
    const double alpha = has(kEpiAlphaDev, g.alpha_dev) ? g.alpha * *g.alpha_dev : g.alpha;
    double shift = g.sq_shift;
    if (has(kEpiShiftDev, g.sq_shift_dev)) shift = *g.sq_shift_dev;
    const double rpx = (has(kEpiRpX, g.rp_x) && col < g.N) ? g.rp_x[col] : 0.0;
    const double qfx = (has(kEpiQf, g.qf_x) && col < g.N) ? g.qf_x[col] : 0.0;
#ifdef VB_GEMM_PROF
    {
      double a_ = alpha, s_ = shift;
      asm volatile("" : "+v"(a_), "+v"(s_), "+v"(r4));
    }
#endif
    VB_GEMM_TS(17);
    // (a two-pass form -- every load first, then every store -- measured no faster:
    // the store phase's ~1 us is the cold instruction cache of this once-per-launch
    // code, 0.3 us when the same stores run a second time; profiles/r04)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i0 + wm * 16 + kq + 4 * r;
      if (row < g.M && col < g.N) {
        double v = alpha * r4[r];
        if (has(kEpiRowDiv, g.row_div)) v = v / g.row_div[row];
        if (has(kEpiColBias, g.col_bias)) v = g.col_bias[col] + v;
        if ((EPI & kEpiDiag) && row == col) v += g.diag;
        double z = 0.0;
        if (is_ns0) {
          const double a = g.A[(long long)row * g.lda + col];
          v = fma(ns0[1], a, ns0[0] * r4[r]);
          z = ns0[2] * ((row == col ? 3.0 : 0.0) - ns0[3] * a);
          g.ns0_z[(long long)row * g.ldc + col] = z;
        }
        double* c = g.C + (long long)row * g.ldc + col;
        if (has(kEpiDot, g.dot_with)) dt = fma(g.dot_with[(long long)row * g.ldc + col], v, dt);
        if (has(kEpiRpX, g.rp_x)) rp[r] = v * rpx;
        if (has(kEpiQf, g.qf_x)) qf = fma(g.qf_x[row] * v, qfx, qf);
        if (has(kEpiRpW, g.rp_w)) rp[r] = v * g.rp_w[(long long)row * g.ldc + col];
        if (has(kEpiBeta, g.beta != 0.0)) v += g.beta * *c;
        *c = v;
        if (mirror) {
          g.C[(long long)col * g.ldc + row] = v;
          if (is_ns0) g.ns0_z[(long long)col * g.ldc + row] = z;
        }
        if constexpr ((EPI & kEpiSq) != 0) {
          const double e = row == col ? v - shift : v;
          sq += e * e;
        }
      }
    }
    VB_GEMM_TS(12);
    const double pw = mirror ? 2.0 : 1.0;   // the transposed tile's share of a sum
    if (has(kEpiSq, g.sq_part)) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off, 64);
      if (lane == 0) g.sq_part[4 * slot + q] = pw * sq;
    }
    if (has(kEpiDot, g.dot_part)) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) dt += __shfl_xor(dt, off, 64);
      if (lane == 0) g.dot_part[4 * slot + q] = pw * dt;
    }
    if (has(kEpiQf, g.qf_part)) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) qf += __shfl_xor(qf, off, 64);
      if (lane == 0) g.qf_part[4 * slot + q] = pw * qf;
    }
    if ((EPI & (kEpiRpX | kEpiRpW)) && (kExact || g.rp_part)) {
      // sum over the 16 lanes of a row (lanes 16 kq .. 16 kq + 15 hold row kq + 4 r)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) rp[r] += __shfl_xor(rp[r], off, 64);
        const int row = i0 + wm * 16 + kq + 4 * r;
        if ((lane & 15) == 0 && row < g.M) g.rp_part[(long long)(2 * bx + wn) * g.M + row] = rp[r];
      }
    }
    VB_GEMM_TS(13);
  }
  __syncthreads();
}

template <bool TA, bool TB, bool KS, bool DUAL, int EPI = kEpiAll>
__global__ __launch_bounds__(NTH) void gemm_f64_kernel(GemmGroup gg) {
  const GemmOp& g = gg.op[blockIdx.z];
#ifndef VB_NO_KWARM
  kernarg_warm(g);   // (every line of the op)
#endif
  __shared__ __attribute__((aligned(16))) double smem[SMEM];
  double(*sA)[BUF] = reinterpret_cast<double(*)[BUF]>(smem);
  double(*sB)[BUF] = reinterpret_cast<double(*)[BUF]>(smem + 2 * BUF);
  VB_GEMM_TS(0);
  int bx = blockIdx.x, by = blockIdx.y, slot = blockIdx.y * gridDim.x + blockIdx.x;
  if ((EPI & kEpiSym) && g.sym) {
    tri_tile(blockIdx.x, (g.N + BT - 1) / BT, by, bx);
    slot = blockIdx.x;
  }
#ifdef VB_GEMM_XCD
  else if (gridDim.x == 16 && gridDim.y == 16) {
    // experiment: block b runs on XCD b % 8 (round-robin dispatch); give XCD x the
    // 4 x 8 rectangle of tiles rows 4 (x / 2) .., columns 8 (x % 2) .., so its L2
    // holds 4 A row panels and 8 B column panels
    const int b = blockIdx.y * 16 + blockIdx.x, x = b & 7, i = b >> 3;
    by = 4 * (x >> 1) + (i >> 3);
    bx = 8 * (x & 1) + (i & 7);
    slot = by * 16 + bx;
  }
#endif
  if (const int sk = gemm_skip<EPI>(g, sB[1])) {
    // the copy decision uses this block's own test (sk == 2) or state written
    // by earlier launches (sk == 1), never a peer block's stores in this launch
    // (launches without copy_src or conv_iter_out never look at the counter)
    bool first = false;
    if (g.copy_src) {
      if (g.copy_if_iter < 0) first = true;
      else if (sk == 2) first = g.conv_iter == g.copy_if_iter;
      else if (g.conv_iter_out) first = *g.conv_iter_out == g.copy_if_iter;
    }
    if (first) {
      for (int e = threadIdx.x; e < BT * BT; e += NTH) {
        const int row = by * BT + e / BT, col = bx * BT + e % BT;
        if (row < g.M && col < g.N) {
          g.C[(long long)row * g.ldc + col] = g.copy_src[(long long)row * g.ldc + col];
          if ((EPI & kEpiSym) && g.sym && bx != by)
            g.C[(long long)col * g.ldc + row] = g.copy_src[(long long)col * g.ldc + row];
        }
      }
    }
    return;
  }
  VB_GEMM_TS(1);
  gemm_tile<TA, TB, KS, DUAL, EPI>(g, bx, by, slot, sA, sB, smem);
  VB_GEMM_TS(15);
}

// Stream-K form of a symmetric pair (gg.op[0], gg.op[1]; both sym, LDS-DMA loop): the
// n_tiles = 2 T upper-triangle tiles x nst k stages of work are dealt over gridDim.x
// blocks, blocks [0, extra) taking base + 1 stages and the rest base, in the order
// (op, tile, stage), nst <= base <= nst (+ 1): a block's stages are the later part of
// one tile (mode 1, or the whole tile) and then the first part of the next (mode 2:
// it finishes that tile with the later part's partial, which the next block computed
// first).  So every block does at most nst + 1 stages instead of 16 CUs running two
// whole tiles (272 tiles on 256 CUs at D = 512).  The skip test and the copy of a
// converged iterate run as in gemm_f64_kernel, the copy dealt by tile (tiles b and
// b + gridDim.x of block b).
template <int EPI>
__global__ __launch_bounds__(NTH) void gemm_f64_sk_kernel(GemmGroup gg, int T, int nst, int base,
                                                          int extra) {
  kernarg_warm(gg);
  __shared__ __attribute__((aligned(16))) double smem[SMEM];
  double(*sA)[BUF] = reinterpret_cast<double(*)[BUF]>(smem);
  double(*sB)[BUF] = reinterpret_cast<double(*)[BUF]>(smem + 2 * BUF);
  const int b = blockIdx.x, nt = (gg.op[0].N + BT - 1) / BT;
  if (const int sk = gemm_skip<EPI>(gg.op[0], sB[1])) {
    for (int tl = b; tl < 2 * T; tl += gridDim.x) {
      const GemmOp& g = gg.op[tl / T];
      bool first = false;
      if (g.copy_src) {
        if (g.copy_if_iter < 0) first = true;
        else if (sk == 2) first = g.conv_iter == g.copy_if_iter;
        else if (g.conv_iter_out) first = *g.conv_iter_out == g.copy_if_iter;
      }
      if (!first) continue;
      int by, bx;
      tri_tile(tl % T, nt, by, bx);
      for (int e = threadIdx.x; e < BT * BT; e += NTH) {
        const int row = by * BT + e / BT, col = bx * BT + e % BT;
        if (row < g.M && col < g.N) {
          g.C[(long long)row * g.ldc + col] = g.copy_src[(long long)row * g.ldc + col];
          if (bx != by) g.C[(long long)col * g.ldc + row] = g.copy_src[(long long)col * g.ldc + row];
        }
      }
    }
    return;
  }
  const int len = b < extra ? base + 1 : base;
  const int u0 = b < extra ? b * (base + 1) : extra * (base + 1) + (b - extra) * base;
  auto run = [&](int tl, int st0, int n, int mode) {
    const GemmOp& g = gg.op[tl / T];
    int by, bx;
    tri_tile(tl % T, nt, by, bx);
    SkPart p;
    p.mode = mode;
    p.st0 = st0;
    p.nst = n;
    p.part = g.sk_part + (long long)tl * (BT * BT);
    p.flag = g.sk_flag + tl;
    p.epoch = g.sk_epoch;
    gemm_tile<false, false, false, false, EPI>(g, bx, by, tl % T, sA, sB, smem, NoHook{}, p);
  };
  // the later stages of tile tA (or all of it), then the first stages of tile tA + 1
  const int tA = u0 / nst, sA0 = u0 % nst, nA = min(nst - sA0, len);
  run(tA, sA0, nA, (sA0 == 0 && nA == nst) ? 0 : 1);
  if (len > nA) {
    const int nB = len - nA;
    run(tA + 1, 0, nB, nB == nst ? 0 : 2);
  }
}

// The same kernel with a hook (see NoHook) built in registers from its
// arguments (Hook(args)); one GemmOp, no skip / copy control (the hook's
// kernels are plain products).
template <bool TA, bool TB, class Hook, int EPI = kEpiAll>
__global__ __launch_bounds__(NTH) void gemm_f64_hook_kernel(GemmGroup gg, typename Hook::Args ha) {
  const GemmOp& g = gg.op[0];
  kernarg_warm(g);
  __shared__ __attribute__((aligned(16))) double smem[SMEM];
  __shared__ __attribute__((aligned(16))) double hlds[Hook::kLds];
  double(*sA)[BUF] = reinterpret_cast<double(*)[BUF]>(smem);
  double(*sB)[BUF] = reinterpret_cast<double(*)[BUF]>(smem + 2 * BUF);
  int bx = blockIdx.x, by = blockIdx.y, slot = blockIdx.y * gridDim.x + blockIdx.x;
  if (g.sym) {
    tri_tile(blockIdx.x, (g.N + BT - 1) / BT, by, bx);
    slot = blockIdx.x;
  }
  gemm_tile<TA, TB, false, false, EPI>(g, bx, by, slot, sA, sB, smem, Hook(ha, slot, hlds));
}

// shape / alignment conditions of the LDS-DMA loop (glds_ok without the A/B switch)
inline bool glds_ok_shape(const GemmOp& o) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return o.M % 32 == 0 && o.N % 32 == 0 && o.K % KTG == 0 && !o.kscale && !o.A2 &&
         o.lda % 2 == 0 && o.ldb % 2 == 0 && al(o.A) && al(o.B);
}

}  // namespace gemm_detail

// The LDS-DMA main loop needs whole 32 x 32 x KTG tiles and 16-byte aligned pairs.
// (gemm_glds_enable: A/B switch for micro-benchmarks; both loops give the same bits)
inline bool gemm_glds_enable = true;
inline bool glds_ok(const GemmOp& o) {
#ifdef VB_GEMM_NO_GLDS
  (void)o;
  return false;
#else
  if (!gemm_glds_enable) return false;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return o.M % 32 == 0 && o.N % 32 == 0 && o.K % gemm_detail::KTG == 0 && !o.kscale && !o.A2 &&
         o.lda % 2 == 0 && o.ldb % 2 == 0 && al(o.A) && al(o.B);
#endif
}

// VIABEL_AMD_GEMM_SYM=0: symmetric results computed in full (A/B switch); callers
// size their partial-sum reductions with gemm_parts
inline bool gemm_sym_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_GEMM_SYM");
    return !(e && e[0] == '0');
  }();
  return on;
}
// VIABEL_AMD_GEMM_EPI_EXACT=0: every launch uses the kEpiAll kernel (A/B switch)
inline bool gemm_epi_exact_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_GEMM_EPI_EXACT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// VIABEL_AMD_GEMM_SK=0: the Newton-Schulz Y|Z pair as one block per tile instead of
// stream-K over one block per CU (A/B switch; the same products, rounded in another
// order where a tile is split)
inline bool gemm_sk_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("VIABEL_AMD_GEMM_SK");
    return !(e && e[0] == '0');
  }();
  return on;
}
// compute units of the current device (stream-K grid), cached per device
inline int gemm_cu_count() {
  static int cached[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cached[dev] = n;
  }
  return cached[dev];
}

namespace gemm_detail {
// The feature set of one op (after gemm_group's sym override), or kEpiAll when a
// feature is half-specified (an exact kernel reads every field of its features).
inline int epi_mask(const GemmOp& o) {
  int m = 0;
  if (o.row_div) m |= kEpiRowDiv;
  if (o.col_bias) m |= kEpiColBias;
  if (o.diag != 0.0) m |= kEpiDiag;
  if (o.ns0) { if (!o.ns0_z) return kEpiAll; m |= kEpiNs0; }
  if (o.dot_with || o.dot_part) { if (!(o.dot_with && o.dot_part)) return kEpiAll; m |= kEpiDot; }
  if (o.rp_x && o.rp_w) return kEpiAll;
  if (o.rp_x || o.rp_w) { if (!o.rp_part) return kEpiAll; m |= o.rp_x ? kEpiRpX : kEpiRpW; }
  else if (o.rp_part) return kEpiAll;
  if (o.qf_x || o.qf_part) { if (!(o.qf_x && o.qf_part)) return kEpiAll; m |= kEpiQf; }
  if (o.beta != 0.0) m |= kEpiBeta;
  if (o.sq_part) m |= kEpiSq;
  if (o.alpha_dev) m |= kEpiAlphaDev;
  if (o.sq_shift_dev) m |= kEpiShiftDev;
  if (o.sym) m |= kEpiSym;
  if (o.skip_flag) m |= kEpiSkip;
  return m;
}
// The feature sets of the full-rank step (vb_fr.hip) that get an exact kernel.
#define VB_GEMM_EPI_SETS(X)                                                        \
  X(0)                                               /* plain products */          \
  X(kEpiSym | kEpiSq)                                /* Sigma = L L^T */           \
  X(kEpiSym | kEpiSq | kEpiQf)                       /* Sigma, with z^T Sigma z */ \
  X(kEpiSym | kEpiNs0)                               /* Newton-Schulz iter 0 */    \
  X(kEpiSym | kEpiAlphaDev | kEpiDiag | kEpiSq | kEpiShiftDev | kEpiSkip) /* T */  \
  X(kEpiSym | kEpiAlphaDev | kEpiSkip)               /* Y | Z */                   \
  X(kEpiDot | kEpiSkip)                              /* PCG Y P, Z R */            \
  X(kEpiAlphaDev | kEpiRowDiv | kEpiColBias)         /* x = mu + c z Y / s */      \
  X(kEpiRpW)                                         /* corr_gauss target */
}  // namespace gemm_detail

// Matrix-core flops of the products this thread has launched (vb_flop_tally):
// per launch, the tiles its grid computes x BT^2 x K x 2 (device-skipped launches
// count too), so a measured step reports the work it ran, not a model
inline double& gemm_flop_tally() {
  static thread_local double t = 0.0;
  return t;
}

// number of 4-per-block partial sums of an n x n result (sym: upper triangle)
inline int gemm_parts(int n, bool sym) {
  const int t = (n + gemm_detail::BT - 1) / gemm_detail::BT;
  return 4 * ((sym && gemm_sym_enabled()) ? t * (t + 1) / 2 : t * t);
}

// Launch n (1 or 2) GEMMs of equal shape and transposes; dual products (A2/B2)
// must not use kscale.
inline hipError_t gemm_group(const GemmOp* ops, int n, hipStream_t s) {
  using namespace gemm_detail;
  const GemmOp& g = ops[0];
  if (g.M <= 0 || g.N <= 0 || n < 1 || n > 2) return n < 1 ? hipSuccess : hipErrorInvalidValue;
  const bool sym_on = gemm_sym_enabled();
  GemmGroup gg{};
  for (int i = 0; i < n; ++i) {
    gg.op[i] = ops[i];
    const GemmOp& o = ops[i];
    gg.op[i].glds = glds_ok(o) ? 1 : 0;
    if (!sym_on) gg.op[i].sym = 0;
  }
  if (gg.op[0].sym && g.M != g.N) return hipErrorInvalidValue;
  // the grid follows op[0]: a group is all-symmetric or all-full, and the row
  // partials (rp_*) are not mirrored into the lower triangle of a sym product
  for (int i = 0; i < n; ++i)
    if (gg.op[i].sym != gg.op[0].sym || (gg.op[i].sym && gg.op[i].rp_part))
      return hipErrorInvalidValue;
  const unsigned ntn = (unsigned)((g.N + BT - 1) / BT);
  const dim3 grid = gg.op[0].sym ? dim3(ntn * (ntn + 1) / 2, 1, (unsigned)n)
                          : dim3(ntn, (unsigned)((g.M + BT - 1) / BT), (unsigned)n);
  const bool ks = g.kscale != nullptr, dual = g.A2 != nullptr;
  if (ks && dual) return hipErrorInvalidValue;
  gemm_flop_tally() += (double)grid.x * grid.y * grid.z * BT * BT * g.K * 2.0 * (dual ? 2 : 1);
  // stream-K for the Newton-Schulz Y|Z pair (GemmOp::sk_part): the tiles' k stages
  // over one block per CU when the tiles outnumber the CUs by at most 1 / nst
  constexpr int kSkEpi = kEpiSym | kEpiAlphaDev | kEpiSkip;
  if (n == 2 && gg.op[0].sk_part && gg.op[1].sk_part && gg.op[0].sym && gg.op[0].glds &&
      gg.op[1].glds && !g.ta && !g.tb && gemm_epi_exact_enabled() && epi_mask(gg.op[0]) == kSkEpi &&
      epi_mask(gg.op[1]) == kSkEpi && gemm_sk_enabled()) {
    const int T = (int)grid.x, nst = g.K / KTG, cus = gemm_cu_count();
    const long long units = 2LL * T * nst;
    if (cus > 0 && 2 * T > cus && units <= (long long)cus * (nst + 1)) {
      const int base = (int)(units / cus), extra = (int)(units % cus);
      hipLaunchKernelGGL((gemm_f64_sk_kernel<kSkEpi>), dim3((unsigned)cus), dim3(NTH), 0, s, gg, T,
                         nst, base, extra);
      return hipGetLastError();
    }
  }
  // exact epilogue kernels: plain NN products whose ops share one listed set, and
  // the NT Sigma = L L^T products (the step's first launch)
  int epi = kEpiAll;
  if (!g.ta && !ks && !dual && gemm_epi_exact_enabled()) {
    epi = epi_mask(gg.op[0]);
    for (int i = 1; i < n; ++i)
      if (epi_mask(gg.op[i]) != epi) epi = kEpiAll;
  }
  if (g.tb && epi != kEpiAll) {
    switch (epi) {
      case kEpiSym | kEpiSq:
        hipLaunchKernelGGL((gemm_f64_kernel<false, true, false, false, kEpiSym | kEpiSq>), grid,
                           dim3(NTH), 0, s, gg);
        return hipGetLastError();
      case kEpiSym | kEpiSq | kEpiQf:
        hipLaunchKernelGGL((gemm_f64_kernel<false, true, false, false, kEpiSym | kEpiSq | kEpiQf>),
                           grid, dim3(NTH), 0, s, gg);
        return hipGetLastError();
      default:
        epi = kEpiAll;
    }
  }
  switch (epi) {
#define VB_EPI_CASE(M)                                                                      \
  case (M):                                                                                 \
    hipLaunchKernelGGL((gemm_f64_kernel<false, false, false, false, (M)>), grid, dim3(NTH), 0, \
                       s, gg);                                                              \
    return hipGetLastError();
    VB_GEMM_EPI_SETS(VB_EPI_CASE)
#undef VB_EPI_CASE
    default:
      break;
  }
#define VB_GEMM(TA, TB)                                                                 \
  do {                                                                                  \
    if (dual)                                                                           \
      hipLaunchKernelGGL((gemm_f64_kernel<TA, TB, false, true>), grid, dim3(NTH), 0, s, gg); \
    else if (ks)                                                                        \
      hipLaunchKernelGGL((gemm_f64_kernel<TA, TB, true, false>), grid, dim3(NTH), 0, s, gg); \
    else                                                                                \
      hipLaunchKernelGGL((gemm_f64_kernel<TA, TB, false, false>), grid, dim3(NTH), 0, s, gg); \
  } while (0)
  if (!g.ta && !g.tb) VB_GEMM(false, false);
  else if (!g.ta && g.tb) VB_GEMM(false, true);
  else if (g.ta && !g.tb) VB_GEMM(true, false);
  else VB_GEMM(true, true);
#undef VB_GEMM
  return hipGetLastError();
}

inline hipError_t gemm(const GemmOp& g, hipStream_t s) { return gemm_group(&g, 1, s); }

// One product (no kscale / dual) with a hook object (gemm_f64_hook_kernel).
template <class Hook>
inline hipError_t gemm_hook(const GemmOp& g0, const typename Hook::Args& hook, hipStream_t s) {
  using namespace gemm_detail;
  if (g0.M <= 0 || g0.N <= 0 || g0.kscale || g0.A2 || g0.skip_flag) return hipErrorInvalidValue;
  if (Hook::kKScale && !glds_ok_shape(g0)) return hipErrorInvalidValue;
  GemmGroup gg{};
  gg.op[0] = g0;
  gg.op[0].glds = (glds_ok(g0) || (Hook::kKScale && glds_ok_shape(g0))) ? 1 : 0;
  if (!gemm_sym_enabled()) gg.op[0].sym = 0;
  if (gg.op[0].sym && (g0.M != g0.N || g0.rp_part)) return hipErrorInvalidValue;
  const unsigned ntn = (unsigned)((g0.N + BT - 1) / BT);
  const dim3 grid = gg.op[0].sym ? dim3(ntn * (ntn + 1) / 2) : dim3(ntn, (unsigned)((g0.M + BT - 1) / BT));
  gemm_flop_tally() += (double)grid.x * grid.y * BT * BT * g0.K * 2.0;
  // the hook's own feature set (Hook::kEpi) when the op matches it exactly
  const bool exact = gemm_epi_exact_enabled() && epi_mask(gg.op[0]) == Hook::kEpi;
  if (!g0.ta && !g0.tb && exact)
    hipLaunchKernelGGL((gemm_f64_hook_kernel<false, false, Hook, Hook::kEpi>), grid, dim3(NTH), 0,
                       s, gg, hook);
  else if (!g0.ta && !g0.tb)
    hipLaunchKernelGGL((gemm_f64_hook_kernel<false, false, Hook>), grid, dim3(NTH), 0, s, gg, hook);
  else if (g0.ta && !g0.tb && exact)
    hipLaunchKernelGGL((gemm_f64_hook_kernel<true, false, Hook, Hook::kEpi>), grid, dim3(NTH), 0,
                       s, gg, hook);
  else if (g0.ta && !g0.tb)
    hipLaunchKernelGGL((gemm_f64_hook_kernel<true, false, Hook>), grid, dim3(NTH), 0, s, gg, hook);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace vbk

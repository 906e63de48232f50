// vb_symsum.hpp — symmetric-sum fp64 MFMA products for the full-rank step's
// conjugate-gradient solve (vb_fr.hip fr_pcg_ss).
//
//   V = A X + X A        A, X symmetric D x D (A: a Newton-Schulz root, X: a CG
//                        vector), D % 64 == 0
//
// V is symmetric, and every block computes COMPLETE entries of it, so the CG's
// vector updates (which need whole entries of V and global scalars from the
// PREVIOUS launch) run in the same block's epilogue: no transposed tile of
// another block is ever needed (a plain product C = A X gives V = C + C^T only
// after a grid-wide dependency, which is what the separate update kernels of
// the old loop waited for).
//
// Blocks (nt = D / 32 tiles a side, nt^2 blocks -- 256 at D = 512, one per CU):
//  * off-diagonal tile (bi < bj), split in two 16-row halves: a half computes
//    rows r0 .. r0 + 15, columns c0 .. c0 + 31 of V as the double-depth product
//      sum_k A[r][k] X[k][c]  +  sum_k X[r][k] A[k][c]        (K = 2 D)
//    and owns those entries (the mirror entries (c, r) are written from them);
//  * diagonal tile (bi == bj): C = A X on the 32 x 32 tile (two 16-row passes,
//    K = D each) and V = C + C^T, symmetrised in LDS.
// Every block does 16 x 32 x 2D MFMA work: the same per-block work as one 32 x 32
// tile of a plain D^3 product, on as many blocks as the plain product's grid.
//
// Main loop: 8 waves = 2 column quadrants (16 x 16) x 4 k parts; operand tiles
// go global -> LDS with LDS-DMA (global_load_lds_dwordx4), 2 stages of KT = 128 k
// (96 KB of dynamic LDS; 64 k, 48 KB, when 128 does not divide D), the next
// stage in flight while one is consumed; each wave reads its A / B
// fragments with inline-asm ds_read_b64 (the compiler cannot tell which DMA a read
// aliases and would wait vmcnt(0) before each) and runs 4 independent
// v_mfma_f64_16x16x4_f64 chains.  Bank-conflict-free layouts as in vb_gemm.hpp:
//   A stage tile: 16 rows x 64 k, slot s of row r holds k = s ^ 2 (r & 15)
//   B stage tile: 64 k x 32 columns, slot s of row k holds column s ^ 16 (k & 1)
#pragma once
#include "vb_device.hpp"
#include "vb_gemm.hpp"

namespace vbk {
namespace symsum {

using d4 = gemm_detail::d4;
// k per LDS stage and stages: KT = 128 x 2 stages (96 KB of dynamic LDS) where D
// allows, else 64 x 2 (48 KB); VB_SS_GS = 3 keeps two stages in flight
// (scripts/ubench/symsum_bench: 11.5 us per 512^3 symmetric sum with 128 x 2,
// 11.8 with 128 x 3, 11.9 / 12.9 with 64 x 3 / 64 x 2; the plain product 9.7)
constexpr int NTH = 512;          // threads per block
constexpr int VS = 33;            // row stride of the result tile in LDS (transposed reads)
constexpr int RED = 3 * 4 * 256;  // k-part reduction scratch (doubles)
#ifndef VB_SS_GS
#define VB_SS_GS 2
#endif
template <int KT>
struct Cfg {
  static constexpr int GS = VB_SS_GS;
  static constexpr int TA = 16 * KT;   // doubles of an A stage tile (16 rows x KT k)
  static constexpr int TB = KT * 32;   // doubles of a B stage tile (KT k x 32 columns)
  static constexpr int ST = TA + TB;
  static constexpr int NA = TA / 1024, NB = TB / 1024;   // DMA instructions per wave and stage
  static constexpr int NS = KT / 16;   // k4 steps per wave and stage (4 k parts)
  static constexpr int LDS_DOUBLES = GS * ST > RED + 2 * 32 * VS ? GS * ST : RED + 2 * 32 * VS;
  static constexpr size_t LDS_BYTES = sizeof(double) * LDS_DOUBLES;
};

// Block geometry: blocks [0, 2 no) are the halves of the no = nt (nt - 1) / 2
// strict-upper tiles (row-major over bi), blocks [2 no, nt^2) the diagonal tiles.
struct Geo {
  int bi, bj, r0, c0;
  bool diag;
};
__host__ __device__ __forceinline__ Geo geo(int b, int nt) {
  const int no = nt * (nt - 1) / 2;
  Geo g;
  if (b < 2 * no) {
    int t = b >> 1, i = 0;
    while (t >= nt - 1 - i) {
      t -= nt - 1 - i;
      ++i;
    }
    g.bi = i;
    g.bj = i + 1 + t;
    g.diag = false;
    g.r0 = 32 * g.bi + 16 * (b & 1);
  } else {
    g.bi = g.bj = b - 2 * no;
    g.diag = true;
    g.r0 = 32 * g.bi;
  }
  g.c0 = 32 * g.bj;
  return g;
}

// The same units in XCD-grouped order.  The dispatcher places block b on XCD b % 8
// (each with its own L2); with nt % 4 == 0 the XCDs take one band block each of the
// 4 x 4 grid of nt/4-tile bands -- (0,1) (0,2) (0,3) (1,2) (1,3) (2,3) -- and the
// diagonal band blocks in pairs, (0,0) + (3,3) and (1,1) + (2,2): nt^2 / 8 units
// each.  An XCD then reads the row and column panels of two bands of each operand
// (1.75-3 MB at D = 512) instead of all of both (4 MB, its whole L2): 11.57 -> 10.77
// us per cold 512^3 symmetric sum (scripts/ubench/symsum_bench.cpp).  Other nt:
// geo()'s order.
__host__ __device__ __forceinline__ Geo geo_xcd(int b, int nt) {
#ifdef VB_SS_NO_XCD
  return geo(b, nt);
#endif
  if (nt % 4 != 0) return geo(b, nt);
  const int x = b & 7, q = b >> 3, m = nt >> 2;
  Geo g;
  if (x < 6) {
    const int ra = x < 3 ? 0 : (x < 5 ? 1 : 2);
    const int cb = x < 3 ? x + 1 : (x < 5 ? x - 1 : 3);
    const int t = q >> 1;
    g.bi = ra * m + t / m;
    g.bj = cb * m + t % m;
    g.diag = false;
    g.r0 = 32 * g.bi + 16 * (q & 1);
  } else {
    const int per = m * m, no = m * (m - 1) / 2;
    const int band = x == 6 ? (q < per ? 0 : 3) : (q < per ? 1 : 2);
    const int u = q < per ? q : q - per;
    if (u < 2 * no) {
      int t = u >> 1, i = 0;
      while (t >= m - 1 - i) {
        t -= m - 1 - i;
        ++i;
      }
      g.bi = band * m + i;
      g.bj = band * m + i + 1 + t;
      g.diag = false;
      g.r0 = 32 * g.bi + 16 * (u & 1);
    } else {
      g.bi = g.bj = band * m + (u - 2 * no);
      g.diag = true;
      g.r0 = 32 * g.bi;
    }
  }
  g.c0 = 32 * g.bj;
  return g;
}

// Entries a block owns: off-diagonal half 16 x 32 (thread t: row t / 32, column
// t % 32), diagonal tile 32 x 32 (thread t: entries t and t + 512).  weight: the
// entry's share of a Frobenius inner product over the whole symmetric matrix.
__device__ __forceinline__ int n_own(const Geo& g) { return g.diag ? 2 : 1; }
__device__ __forceinline__ double own_weight(const Geo& g) { return g.diag ? 1.0 : 2.0; }

// V of the block into vt (rows 0..15 or 0..31, stride VS), unscaled: entries of
// A X + X A.  lds: Cfg<KT>::LDS_DOUBLES of dynamic LDS; vt = lds + RED.  Ends with
// a barrier (vt complete; the stage buffers are free again).  go() is asked after
// the first stage is issued (its loads in flight): false (the same in every wave
// of the block) drains them and returns false before any barrier.
#ifdef VB_SS_PROF
// phase stamps of the calling thread (s_memrealtime, 100 MHz): first stage landed,
// main loop done
#define VB_SS_STAMPS , unsigned long long* vb_ss_stamp
#else
#define VB_SS_STAMPS
#endif
template <int KT, class Go>
__device__ __forceinline__ bool product(const double* __restrict__ Am, const double* __restrict__ Xm,
                                        int D, const Geo& g, double* lds, Go&& go VB_SS_STAMPS) {
  using C = Cfg<KT>;
  constexpr int GS = C::GS, TA = C::TA, ST = C::ST, NA = C::NA, NB = C::NB, NS = C::NS;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wn = w & 1, h = w >> 1, kq = lane >> 4;
  const int NT1 = D / KT, nst = 2 * NT1;
  // per-lane DMA sources within a stage tile (element offsets from its origin);
  // DMA instruction j of wave w fills LDS doubles [128 (8 j + w), + 128)
  long long aoff[NA], boff[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int o = 128 * (8 * j + w) + 2 * lane, r = o / KT, s = o % KT;
    aoff[j] = (long long)r * D + (s ^ (2 * (r & 15)));
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int o = 128 * (8 * j + w) + 2 * lane, r = o >> 5, s = o & 31;
    boff[j] = (long long)r * D + (s ^ (16 * (r & 1)));
  }
  // stage it: k block (it mod NT1); off-diagonal halves switch operands (A X, then
  // X A) at it = NT1, diagonal tiles switch rows (the tile's second 16-row pass)
  auto issue = [&](int it, int slot) {
    const bool second = it >= NT1;
    const int k0 = (second ? it - NT1 : it) * KT;
    const double* a = (second && !g.diag) ? Xm : Am;
    const double* b = (second && !g.diag) ? Am : Xm;
    const int r0 = g.r0 + ((second && g.diag) ? 16 : 0);
    a += (long long)r0 * D + k0;
    b += (long long)k0 * D + g.c0;
    double* st = lds + slot * ST;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(a + aoff[j]), (void*)(st + 128 * (8 * j + w)),
                                       16, 0, 0);
#pragma unroll
    for (int j = 0; j < NB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(b + boff[j]),
                                       (void*)(st + TA + 128 * (8 * j + w)), 16, 0, 0);
  };
  typedef __attribute__((address_space(3))) double lds_f64;
  const unsigned la = (unsigned)(uintptr_t)((lds_f64*)lds);
  const int ar = lane & 15, bc = 16 * wn + (lane & 15);
  unsigned xa[NS], xb[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = (KT / 4) * h + 4 * s + kq;
    xa[s] = la + 8u * (unsigned)(ar * KT + (k ^ (2 * ar)));
    xb[s] = la + 8u * (unsigned)(TA + k * 32 + (bc ^ (16 * (k & 1))));
  }
  d4 acc[4], top = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
  issue(0, 0);
  if (GS >= 3 && nst > 1) issue(1, 1);
  if (!go()) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return false;
  }
  // stage it's buffer, and the buffer of the stage issued after its barrier
  int slot = 0, slot2 = GS >= 3 ? 2 : 1;
  for (int it = 0; it < nst; ++it) {
    // stage it landed (this wave's DMAs; the barrier covers the other waves'),
    // the buffer consumed at it - 1 is free for stage it + 2
    if (GS >= 3 && it + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA + NB) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#ifdef VB_SS_PROF
    if (it == 0) vb_ss_stamp[0] = __builtin_amdgcn_s_memrealtime();
#endif
    if (it + GS - 1 < nst) issue(it + GS - 1, slot2);
    if (g.diag && it == NT1) {   // the tile's first 16 rows are done
      top = (acc[0] + acc[1]) + (acc[2] + acc[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
    }
    const unsigned so = (unsigned)(slot * ST * 8);
    // four steps' reads in flight; step s + 4 is read after step s's MFMA
    double fa[NS], fb[NS];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      asm volatile("ds_read_b64 %0, %1" : "=v"(fa[s]) : "v"(xa[s] + so));
      asm volatile("ds_read_b64 %0, %1" : "=v"(fb[s]) : "v"(xb[s] + so));
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int ahead = (NS - 1 - s) < 3 ? (NS - 1 - s) : 3;
      if (ahead == 3) asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(fa[s]), "+v"(fb[s]));
      else if (ahead == 2) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(fa[s]), "+v"(fb[s]));
      else if (ahead == 1) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(fa[s]), "+v"(fb[s]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[s]), "+v"(fb[s]));
      acc[s & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[s], fb[s], acc[s & 3], 0, 0, 0);
// (rejected: the next stage's DMA pieces one per MFMA step: 12.05 vs 11.50 us)
      if (s + 4 < NS) {
        asm volatile("ds_read_b64 %0, %1" : "=v"(fa[s + 4]) : "v"(xa[s + 4] + so));
        asm volatile("ds_read_b64 %0, %1" : "=v"(fb[s + 4]) : "v"(xb[s + 4] + so));
      }
    }
    slot = slot + 1 == GS ? 0 : slot + 1;
    slot2 = slot2 + 1 == GS ? 0 : slot2 + 1;
  }
#ifdef VB_SS_PROF
  vb_ss_stamp[1] = __builtin_amdgcn_s_memrealtime();
#endif
  const d4 r4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  // k parts 1..3 hand their quadrants to part 0 through LDS (fixed order)
  __syncthreads();
  double* red = lds;
  double* vt = lds + RED;
  const int nh = g.diag ? 2 : 1;
  if (h >= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      red[(((h - 1) * 2 + 0) * 2 + wn) * 256 + r * 64 + lane] = g.diag ? top[r] : r4[r];
      if (g.diag) red[(((h - 1) * 2 + 1) * 2 + wn) * 256 + r * 64 + lane] = r4[r];
    }
  }
  __syncthreads();
  if (h == 0) {
    for (int hf = 0; hf < nh; ++hf) {
      const d4 own = (g.diag && hf == 0) ? top : r4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double p1 = red[((0 * 2 + hf) * 2 + wn) * 256 + r * 64 + lane];
        const double p2 = red[((1 * 2 + hf) * 2 + wn) * 256 + r * 64 + lane];
        const double p3 = red[((2 * 2 + hf) * 2 + wn) * 256 + r * 64 + lane];
        vt[(16 * hf + kq + 4 * r) * VS + 16 * wn + (lane & 15)] = (own[r] + p1) + (p2 + p3);
      }
    }
  }
  __syncthreads();
  if (g.diag) {   // V = C + C^T on the diagonal tile (each pair by one thread)
    for (int e = t; e < 32 * 32; e += NTH) {
      const int r = e >> 5, c = e & 31;
      if (r < c) {
        const double s = vt[r * VS + c] + vt[c * VS + r];
        vt[r * VS + c] = s;
        vt[c * VS + r] = s;
      } else if (r == c) {
        vt[r * VS + r] = 2.0 * vt[r * VS + r];
      }
    }
    __syncthreads();
  }
  return true;
}
template <int KT>
__device__ __forceinline__ void product(const double* __restrict__ Am, const double* __restrict__ Xm,
                                        int D, const Geo& g, double* lds) {
#ifdef VB_SS_PROF
  unsigned long long st[2];
  product<KT>(Am, Xm, D, g, lds, [] { return true; }, st);
#else
  product<KT>(Am, Xm, D, g, lds, [] { return true; });
#endif
}

// Block sum of one value per thread (fixed order: DPP wave sums, then the 8 waves
// in order); every thread gets the total.  scratch: 8 doubles of LDS.
__device__ __forceinline__ double block_sum8(double v, double* scratch) {
  v = vbd::wave_sum_dpp(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  const double s = ((scratch[0] + scratch[1]) + (scratch[2] + scratch[3])) +
                   ((scratch[4] + scratch[5]) + (scratch[6] + scratch[7]));
  __syncthreads();
  return s;
}

// Block sums of NV values per thread at once (one LDS exchange, two barriers):
// each v[j] becomes its block total, in block_sum8's fixed order.  scratch: 8 NV
// doubles of LDS.
template <int NV>
__device__ __forceinline__ void block_sum8v(double (&v)[NV], double* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    v[j] = vbd::wave_sum_dpp(v[j]);
    if (lane == 0) scratch[8 * j + w] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const double* q = scratch + 8 * j;
    v[j] = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  }
  __syncthreads();
}

// Plain symmetric-sum product C = alpha (A X + X A) (measurement / tests).
template <int KT>
__global__ __launch_bounds__(NTH) void symsum_plain_kernel(const double* A, const double* X, int D,
                                                           double alpha, double* C) {
  extern __shared__ double lds[];
  const Geo g = geo_xcd(blockIdx.x, D / 32);
  product<KT>(A, X, D, g, lds);
  const double* vt = lds + RED;
  const int t = threadIdx.x;
  for (int e = t; e < (g.diag ? 1024 : 512); e += NTH) {
    const int r = e >> 5, c = e & 31;
    C[(long long)(g.r0 + r) * D + g.c0 + c] = alpha * vt[r * VS + c];
  }
  if (!g.diag) {   // mirror: thread t -> (column c, row r) of the transposed half
    const int c = t >> 4, r = t & 15;
    C[(long long)(g.c0 + c) * D + g.r0 + r] = alpha * vt[r * VS + c];
  }
}

inline bool usable(int D, const void* a, const void* x) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return D >= 64 && D % 64 == 0 && al(a) && al(x);
}
// the stage depth for D (128 where it divides D)
inline int kt_for(int D) { return D % 128 == 0 ? 128 : 64; }

inline hipError_t plain(const double* A, const double* X, int D, double alpha, double* C,
                        hipStream_t s, int kt = 0) {
  if (!usable(D, A, X)) return hipErrorInvalidValue;
  if (kt == 0) kt = kt_for(D);
  if (D % kt) return hipErrorInvalidValue;
  const int nt = D / 32;
  if (kt == 128)
    hipLaunchKernelGGL(symsum_plain_kernel<128>, dim3(nt * nt), dim3(NTH), Cfg<128>::LDS_BYTES, s, A,
                       X, D, alpha, C);
  else
    hipLaunchKernelGGL(symsum_plain_kernel<64>, dim3(nt * nt), dim3(NTH), Cfg<64>::LDS_BYTES, s, A, X,
                       D, alpha, C);
  return hipGetLastError();
}

}  // namespace symsum
}  // namespace vbk

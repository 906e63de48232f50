// vb_gemm_comb.hpp — the preconditioned-CG GEMMs of the sqrtm VJP (vb_fr.hip
// fr_pcg) with the CG vector updates folded into the operand loads.
//
// One CG iteration used to be four launches: C1 = Y P, then an elementwise
// kernel (X += alpha P, R -= alpha (C1 + C1^T)), C2 = Z R, then another
// (P = (C2 + C2^T) / 4 + beta P).  The updates need alpha / beta, i.e. global
// inner products of the previous GEMM's output, so they cannot ride in that
// GEMM's epilogue -- but they are linear, so the NEXT GEMM can form its own B
// operand on the fly:
//   ZR:  B = R_it - alpha (C1 + C1^T)       = R_{it+1},  C2 = Z R_{it+1}
//   YP:  B = beta P_{it-1} + (C2 + C2^T) / 4 = P_it,     C1 = Y P_it
// Every block sums the partial inner products itself (same order everywhere)
// to get alpha / beta, streams R (or P), C and the transposed tile of C
// through LDS-DMA, and combines the three fragments in registers before each
// MFMA.  The block whose k tile equals its row tile writes the combined tile
// (the CG vector for the next launch: each element written once); the
// epilogue forms <B, C> and ||B||^2 partials from that tile and, for ZR, the
// elementwise X += alpha P of its output tile.  Two launches per iteration.
//
// Shapes: D x D row-major, D a multiple of 32 (the LDS-DMA tiles of vb_gemm.hpp).
#pragma once
#include "vb_gemm.hpp"

namespace vbk {

struct CombOp {
  int D;
  int mode;               // 0: ZR init (B = R_0), 1: ZR, 2: YP
  int it;                 // CG iteration
  const double* A;        // Z (ZR) or Y (YP)
  const double* B0;       // ZR: R_it;  YP: P_{it-1} (it >= 1)
  const double* B1;       // ZR: C1 = Y P_it;  YP: C2 = Z R_it
  double* Bout;           // ZR: R_{it+1};  YP: P_it (mode 0: not written)
  double* C;              // ZR: C2;  YP: C1
  const double* rz_new;   // partials of <R_it, C2_prev> (rz_it = sum / 2)
  const double* rz_old;   // YP, it >= 1: partials of rz_{it-1}
  int n_rz;
  const double* pq;       // ZR: partials of <P_it, C1> (alpha = rz_it / (2 sum))
  int n_pq;
  double* dot_out;        // partials of <B, C> over this block's tile (4 per block)
  double* rr_out;         // ZR: ||R_{it+1}||^2 partial (1 per block)
  double* X;              // ZR: X = (it == 0 ? 0 : X) + alpha P_it
  const double* P;        // ZR: P_it
  int* done;              // CG converged (set by a YP test; later launches return)
  const double* rr_in;    // YP, it >= 1: ||R_it||^2 partials ...
  int n_rr;
  const double* ee_part;  // ... converged when sum <= tol2 * sum(ee_part) (= ||E||^2)
  int n_ee;
  double* ee_out;         // YP, it == 0: block (0, 0) stores ||E||^2 (the status check's scale)
  double tol2;
  int* conv_iter_out;     // YP: it - 1 at convergence (the last update needed)
};

namespace gemm_detail {

constexpr int CGS = 3;                 // LDS stages of the combined loop
constexpr int CSRC = 4;                // tiles per stage: A, B0, B1, B1^T
constexpr int CSMEM = CGS * CSRC * TD + TD + 64;

__device__ __forceinline__ double block_sum_fixed(const double* p, int n, double* red) {
  // every block of the launch sums the same partials in the same order
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += NTH) a += p[i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) a += __shfl_xor(a, off, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < NTH / 64; ++k) t += red[k];
  return t;
}

__global__ __launch_bounds__(NTH) void gemm_comb_kernel(CombOp o) {
  static_assert(GKT == KT && GPW == 1, "combined CG loop: 32-deep tiles, one LDS-DMA per wave");
  __shared__ __attribute__((aligned(16))) double smem[CSMEM];
  __shared__ int s_skip;
  double* red = smem + CGS * CSRC * TD + TD;   // 64 doubles of scratch
  double* sBo = smem + CGS * CSRC * TD;        // the combined tile [k][col] (k tile == row tile)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = w & 3, h = w >> 2, wm = q >> 1, wn = q & 1, kq = lane >> 4;
  const int D = o.D, bx = blockIdx.x, by = blockIdx.y;
  const int i0 = by * BT, j0 = bx * BT;
  // ---- skip / convergence test (state of earlier launches only) -------------
  if (t == 0) s_skip = __hip_atomic_load(o.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  __syncthreads();
  if (s_skip) return;
  if (o.mode == 2 && o.it == 0 && bx == 0 && by == 0) {
    const double ee = block_sum_fixed(o.ee_part, o.n_ee, red);
    if (t == 0) *o.ee_out = ee;
  }
  if (o.mode == 2 && o.it >= 1) {
    const double rr = block_sum_fixed(o.rr_in, o.n_rr, red);
    const double ee = block_sum_fixed(o.ee_part, o.n_ee, red);
    if (rr <= o.tol2 * ee) {
      if (t == 0) {
        *o.conv_iter_out = o.it - 1;
        __hip_atomic_store(o.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  // ---- coefficients: B = c0 B0 + c1 (B1 + B1^T) -------------------------------
  double c0 = 1.0, c1 = 0.0, alpha = 0.0;
  if (o.mode == 1) {
    const double rz = 0.5 * block_sum_fixed(o.rz_new, o.n_rz, red);
    const double pq = block_sum_fixed(o.pq, o.n_pq, red);
    alpha = rz / (2.0 * pq);
    c1 = -alpha;
  } else if (o.mode == 2) {
    c1 = 0.25;
    c0 = 0.0;
    if (o.it >= 1) {
      const double rz = 0.5 * block_sum_fixed(o.rz_new, o.n_rz, red);
      const double rzo = 0.5 * block_sum_fixed(o.rz_old, o.n_rz, red);
      c0 = rz / rzo;
    }
  }
  const bool use_b0 = o.mode != 2 || o.it >= 1;
  const bool use_b1 = o.mode != 0;
  // ---- main loop: LDS-DMA of A, B0, B1 (rows = k) and B1^T (rows = n) --------
  const long long ld = D;
  const double* a0 = o.A + (long long)i0 * ld;
  const double* p0 = o.B0 + j0;
  const double* p1 = o.B1 + j0;
  const double* p1t = o.B1 + (long long)j0 * ld;
  const long long aoff = glds_src<true>(w, lane, ld), boff = glds_src<false>(w, lane, ld);
  const int nt = D / KT;
  auto issue = [&](int it) {
    double* st = smem + (it % CGS) * CSRC * TD + 128 * w;
    __builtin_amdgcn_global_load_lds((const void*)(a0 + it * KT + aoff), (void*)st, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(p0 + (long long)it * KT * ld + boff),
                                     (void*)(st + TD), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(p1 + (long long)it * KT * ld + boff),
                                     (void*)(st + 2 * TD), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(p1t + it * KT + aoff), (void*)(st + 3 * TD),
                                     16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < CGS - 1; ++s)
    if (s < nt) issue(s);
  const int ra = wm * 16 + (lane & 15), cb = wn * 16 + (lane & 15);
  typedef __attribute__((address_space(3))) double lds_f64;
  const unsigned base = (unsigned)(uintptr_t)((lds_f64*)smem);
  unsigned xa[4], xb[4], xt[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int kk = h * (KT / KS_) + 4 * s + kq;
    xa[s] = base + 8u * (unsigned)glds_at<true>(ra, kk);
    xb[s] = base + 8u * (unsigned)(TD + glds_at<false>(kk, cb));
    xt[s] = base + 8u * (unsigned)(3 * TD + glds_at<true>(cb, kk));
  }
  d4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
  constexpr unsigned B1OFF = 8u * TD;  // B1 tile: one tile after B0 (same layout)
  for (int it = 0; it < nt; ++it) {
    const int last_issued = it + CGS - 2 < nt - 1 ? it + CGS - 2 : nt - 1;
    const int pending = last_issued - it;
    if (pending >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it + CGS - 1 < nt) issue(it + CGS - 1);
    const unsigned so = (unsigned)((it % CGS) * CSRC * TD * 8);
    const bool wr = it == by && wm == 0;   // this wave writes the combined tile
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      double a, b0, b1, bt;
      asm volatile("ds_read_b64 %0, %1" : "=v"(a) : "v"(xa[s] + so));
      asm volatile("ds_read_b64 %0, %1" : "=v"(b0) : "v"(xb[s] + so));
      asm volatile("ds_read_b64 %0, %1" : "=v"(b1) : "v"(xb[s] + so + B1OFF));
      asm volatile("ds_read_b64 %0, %1" : "=v"(bt) : "v"(xt[s] + so));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b0), "+v"(b1), "+v"(bt));
      const double sym = use_b1 ? b1 + bt : 0.0;
      double b = use_b0 ? fma(c1, sym, c0 * b0) : c1 * sym;
      if (o.mode == 1) b = fma(c1, sym, b0);       // R - alpha (C1 + C1^T)
      if (wr) {
        const int k = h * (KT / KS_) + 4 * s + kq;
        sBo[k * BT + cb] = b;
        if (o.mode != 0) o.Bout[(long long)(i0 + k) * ld + j0 + cb] = b;
      }
      acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[s], 0, 0, 0);
    }
  }
  __syncthreads();
  // ---- epilogue: k parts -> part 0, then C, <B, C>, ||B||^2, X update --------
  d4 r4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  double* rbuf = smem;   // the stages are free now
  if (h >= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rbuf[(q * 4 + r) * 64 + lane] = r4[r];
  }
  __syncthreads();
  if (h == 0) {
    const int col = wn * 16 + (lane & 15);
    double dt = 0.0, sq = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wm * 16 + kq + 4 * r;
      const double v = r4[r] + rbuf[(q * 4 + r) * 64 + lane];
      const long long idx = (long long)(i0 + row) * ld + j0 + col;
      o.C[idx] = v;
      const double bv = sBo[row * BT + col];
      dt = fma(bv, v, dt);
      sq = fma(bv, bv, sq);
      if (o.mode == 1) o.X[idx] = fma(alpha, o.P[idx], o.it == 0 ? 0.0 : o.X[idx]);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      dt += __shfl_xor(dt, off, 64);
      sq += __shfl_xor(sq, off, 64);
    }
    if (lane == 0) {
      o.dot_out[4 * (by * gridDim.x + bx) + q] = dt;
      red[q] = sq;
    }
  }
  __syncthreads();
  if (o.mode == 1 && t == 0)
    o.rr_out[by * gridDim.x + bx] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace gemm_detail

inline hipError_t gemm_comb(const CombOp& o, hipStream_t s) {
  if (o.D <= 0 || o.D % 32 != 0) return hipErrorInvalidValue;
  const unsigned nb = (unsigned)(o.D / 32);
  hipLaunchKernelGGL(gemm_detail::gemm_comb_kernel, dim3(nb, nb), dim3(gemm_detail::NTH), 0, s, o);
  return hipGetLastError();
}

}  // namespace vbk

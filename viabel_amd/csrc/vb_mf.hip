// vb_mf.hip — mean-field Gaussian / Student-t Monte Carlo VI kernels for gfx950.
//
// Reference path (paths relative to the reference repo):
//   families       viabel/vb.py:48-82, 140-182
//   KLVI           viabel/vb.py:236-245      value = -(H(lam) + mean_n log p(x_n))
//   CHIVI          viabel/vb.py:248-266      value = log(mean w)/alpha + max lw,
//                                            grad  = alpha/N sum_n w_n d lw_n / d lam
//   adagrad        viabel/vb.py:345-389      windowed adagrad, tail-quarter history
//
// Two kernel shapes:
//  * sep_kernel    one wavefront owns a column pair (d, d+1) of a SEPARABLE target
//                  and all N samples of it, for every step of a chunk: the
//                  mean-field KLVI objective, its gradient and the adagrad update
//                  of those four parameters never need another column, so the
//                  whole optimisation runs in registers with no inter-wave
//                  traffic.  Noise is regenerated from Philox counters, never
//                  stored; HBM sees only per-step value partials and history rows.
//  * block_kernel  one workgroup owns one problem (restart) of dimension
//                  D <= kBlockDMax with any target, KLVI or CHIVI; samples are
//                  spread over the 256 threads, reductions go wave-shuffle -> LDS.
#include "vb_device.hpp"
#include "vb_internal.hpp"

#include <cstdlib>
#include <type_traits>
#include <utility>

using namespace vbd;

namespace vbk {

// -------------------------------------------------------------------------
// column-pair persistent KLVI kernel
// -------------------------------------------------------------------------
// DPP move with an undefined "old" operand.  Every control used by the
// column-pair kernel (quad_perm, row_ror, row_newbcast) reads a lane of the same
// row, and the kernel reduces with all 64 lanes active, so "old" is never
// selected: leaving it undefined spares the v_mov that would initialise it.
template <int CTRL>
__device__ __forceinline__ double dppu_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Sum over the 16 lanes of each DPP row.  Pairwise symmetric steps (xor 1,
// xor 2, half mirror, mirror): every lane of the row gets the bitwise-identical
// total, so the owner lanes of a parameter evolve it identically.
__device__ __forceinline__ double row_sum16(double v) {
  v += dppu_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dppu_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dppu_f64<0x141>(v);  // row_half_mirror
  return v + dppu_f64<0x140>(v);  // row_mirror
}

// Sum over lanes l = c (mod 4) of a group of 64/PPW lanes (PPW >= 2).
template <int PPW>
__device__ __forceinline__ double stride4_sumu(double k) {
  k += dppu_f64<0x124>(k);  // row_ror:4
  k += dppu_f64<0x128>(k);  // row_ror:8
  if constexpr (PPW == 2) k = swap_sum16(k);  // rows 0+1, 2+3
  return k;
}

// Permlane swaps of two different quantities x, y (no copies needed): the sum
// of the swapped registers is a reduce-scatter over row pairs (swap16: rows
// 0+1 of x land in row 0, of y in row 1, ...) or wave halves (swap32).
__device__ __forceinline__ double swap16_rs(double x, double y) {
  const auto a = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(x),
                                                  (unsigned)__double2loint(y), false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x),
                                                  (unsigned)__double2hiint(y), false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
__device__ __forceinline__ double swap32_rs(double x, double y) {
  const auto a = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(x),
                                                  (unsigned)__double2loint(y), false, false);
  const auto b = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(x),
                                                  (unsigned)__double2hiint(y), false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}

// Reduce-scatter of four per-lane partial sums (q0..q3) over the LPP = 64 / PPW
// lanes of one column pair; the lane's "owner" quantity total is returned
// (sep_owner below says which lane owns which quantity).
//  * PPW >= 2: lane l owns quantity l & 3.  Two DPP exchange steps hand each
//    lane one quantity; two row rotations and, for 2-row groups, a permlane
//    swap finish the sum.
//  * PPW == 1: row r owns quantity r.  Two permlane16 swaps of (q0, q1) and
//    (q2, q3) and one permlane32 swap scatter the quantities over the rows (no
//    register copies: the swapped operands are different quantities), then a
//    16-lane row sum.
template <int PPW>
__device__ __forceinline__ double reduce4(int lane, double q0, double q1, double q2, double q3) {
  if constexpr (PPW == 1) {
    return row_sum16(swap32_rs(swap16_rs(q0, q1), swap16_rs(q2, q3)));
  } else {
    const bool b0 = lane & 1, b1 = lane & 2;
    double kg = b0 ? q1 : q0, kh = b0 ? q3 : q2;
    kg += dppu_f64<0xB1>(b0 ? q0 : q1);  // quad_perm [1,0,3,2]: partner keeps the other column
    kh += dppu_f64<0xB1>(b0 ? q2 : q3);
    double k = b1 ? kh : kg;
    k += dppu_f64<0x4E>(b1 ? kg : kh);   // quad_perm [2,3,0,1]
    return stride4_sumu<PPW>(k);
  }
}

// Sum over the lanes that hold one parameter's window slots: the 16 lanes of
// its row (PPW == 1) or the residue class l & 3 of its group (PPW >= 2).
template <int PPW>
__device__ __forceinline__ double owner_sum(double v) {
  if constexpr (PPW == 1) return row_sum16(v);
  else return stride4_sumu<PPW>(v);
}

// Value held by the owner lane of quantity K, for every lane of the group.
// 4 pairs per wave: a group is one DPP row, so row_newbcast:K (dpp_ctrl 0x150 +
// K) does it; 2 pairs: newbcast, then permlane16_swap copies each even row into
// the odd row above it; 1 pair: readlane of row K's first lane (wave-uniform).
template <int PPW, int K>
__device__ __forceinline__ double group_bcast(double v, int /*grp*/) {
  if constexpr (PPW == 1) {
    return readlane_f64(v, 16 * K);
  } else {
    const double t = dppu_f64<0x150 + K>(v);
    if constexpr (PPW == 4) {
      return t;
    } else {
      const unsigned lo = (unsigned)__double2loint(t), hi = (unsigned)__double2hiint(t);
      const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
      const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
      return __hiloint2double((int)b[0], (int)a[0]);
    }
  }
}

// 1 / sqrt(y), y > 0: v_rsq_f64 seed + two Newton steps (~1 ulp).
__device__ __forceinline__ double rsqrt_pos(double y) {
  double r = __builtin_amdgcn_rsq(y);
  const double hy = 0.5 * y;
  r = r * fma(-hy * r, r, 1.5);
  r = r * fma(-hy * r, r, 1.5);
  return r;
}

// PPW column pairs per wavefront (PPW in {1, 2, 4}); pair = wave * PPW + lane / LPP.
// Owner lanes: quantity / parameter q (0 muA, 1 muB, 2 log sA, 3 log sB) is
// owned by lane q of the group (PPW >= 2) or by every lane of row q (PPW == 1,
// whose rep lane 16 q updates it); see reduce4.
// REGRING: the adagrad window (W <= 16) lives in registers, one entry per
// (lane, j) among the SL lanes that own the parameter: slot j * SL + sub;
// otherwise in LDS.
// Per-step values: each lane keeps the last four steps' partial values in
// registers and one reduce-scatter every fourth step sums all four (the
// entropy term sum log s rides in the partial of the log-scale rep lanes).
#ifdef VB_SEP_TS
// per-wave step timestamps of the launch whose first step is VB_SEP_TS (slot =
// blockIdx.x * 4 + wave; [0] step 0 ... [k] step 2^(k-1), [13] last step,
// [14] PPW, [15] kernel entry), read back by vb_debug_sep_ts
constexpr int kTsWaves = 8192;
__device__ unsigned long long g_sep_ts[kTsWaves][16];
__device__ unsigned long long g_sep_clk[kTsWaves][16];  // s_memtime (core clock) beside it
#endif

// lambda and the register window of a wave's owner lanes, loaded before the
// kernel's table barrier (the loads then overlap the table loads instead of
// following them; sep_body's lane mapping)
template <int PPW>
struct SepPre {
  double lam = 0.0;
  double rg[PPW] = {};
};
template <int PPW, bool REGRING, bool ADV = false>
__device__ __forceinline__ SepPre<PPW> sep_pre(const SepArgs& a, int wave) {
  constexpr int LPP = 64 / PPW, SL = LPP / 4;
  const int lane = threadIdx.x & 63, grp = lane / LPP, gl = lane & (LPP - 1);
  const int w = wave * PPW + grp, D = a.D;
  const bool live = w < a.n_pairs, hasB = live && 2 * w + 1 < D;
  const int own = PPW == 1 ? lane >> 4 : lane & 3;
  const int sub = PPW == 1 ? lane & 15 : gl >> 2;
  const long long own_idx = (own & 2 ? D : 0) + (own & 1 ? 2 * w + 1 : 2 * w);
  const bool own_ok = live && (hasB || !(own & 1));
  SepPre<PPW> p;
  p.lam = own_ok ? a.lam[own_idx] : 0.0;
  if constexpr (REGRING) {
    if (ADV || !a.emit_grad) {
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int sl = j * SL + sub;
        if (sl < a.W && own_ok) p.rg[j] = a.ring[(long long)sl * 2LL * D + own_idx];
      }
    }
  }
  return p;
}

template <class TGT, bool TFAM, bool HOST, int PPW, bool REGRING, bool ADV = false>
__device__ __forceinline__ void sep_body(const SepArgs& a, double* ring_base, int wave,
                                         const double2* sct, const double2* ltab,
                                         const SepPre<PPW>& pre, unsigned long long t_entry = 0) {
  constexpr int LPP = 64 / PPW;       // lanes per column pair
  constexpr int SL = LPP / 4;         // slot lanes per parameter
#ifdef VB_SEP_PROF
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
  const int lane = threadIdx.x & 63;
  const int grp = lane / LPP;
  const int gl = lane & (LPP - 1);    // lane within the pair's group
  const int w = wave * PPW + grp;     // column pair of this lane
  const bool live = w < a.n_pairs;    // trailing groups of the last wave may be empty
  const int D = a.D, N = a.N, W = a.W;
  // ADV: the optimisation launches (vb_run_advance) -- no emitted gradient and the
  // plain KLVI value -- as compile-time constants, so the step loop carries no branch,
  // mask or scalar reload for the single-call forms (the headline's launches)
  const int emit_grad = ADV ? 0 : a.emit_grad;
  const int pdv = ADV ? 0 : a.pd;
  const long long P = 2LL * D;
  const int dA = 2 * w, dB = 2 * w + 1;
  const bool hasB = live && dB < D;
  const double hbw = hasB ? 1.0 : 0.0;   // (the separable targets' lp1 is finite)
  // isotropic Gaussian target: the log p constant of the rows this lane consumes per
  // step (rows gl, gl + LPP, ... below N)
  constexpr bool kQuad = std::is_same_v<TGT, IsoGauss>;
  const double quad_c = -0.5 * kLog2Pi * (double)(gl < N ? (N - 1 - gl) / LPP + 1 : 0);
  double* ring = ring_base + grp * 4;  // LDS ring [slot][PPW * 4]

  const int own = PPW == 1 ? lane >> 4 : lane & 3;        // 0 muA, 1 muB, 2 lsA, 3 lsB
  const int sub = PPW == 1 ? lane & 15 : gl >> 2;         // index among the owner lanes
  const bool rep = sub == 0;                              // the owner lane that writes
  const long long own_idx = (own & 2 ? D : 0) + (own & 1 ? dB : dA);
  const bool own_ok = live && (hasB || !(own & 1));
  const bool updater = rep && own_ok;
  double lam_own = pre.lam;
  double s_own = exp_fast(lam_own);
  double muA = group_bcast<PPW, 0>(lam_own, grp), muB = group_bcast<PPW, 1>(lam_own, grp);
  double sA = group_bcast<PPW, 2>(s_own, grp), sB = group_bcast<PPW, 3>(s_own, grp);

  int slot = 0, cnt = 0;
  double rg[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) rg[j] = 0.0;
  if (!emit_grad) {
    if constexpr (REGRING) {
#pragma unroll
      for (int j = 0; j < PPW; ++j) rg[j] = pre.rg[j];
    } else {
      if (rep)
        for (int k = 0; k < W; ++k)
          ring[k * 4 * PPW + own] = own_ok ? a.ring[(long long)k * P + own_idx] : 0.0;
    }
    slot = (int)(a.step0 % W);
    cnt = a.step0 < W ? (int)a.step0 : W;
  }
  const Rng rng{a.k0, a.k1, a.stream};
  const double invN = 1.0 / (double)N;
  // entropy share of this lane's value partial: log s of its rep lane
  const bool ent = updater && own >= 2;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;  // partials of steps s, s-1, s-2, s-3
  // Philox Gaussian draws: the first sample row of each step is drawn one step
  // ahead (software pipelining across the step boundary)
  constexpr bool PIPE = !HOST && !TFAM;
  double pA = 0.0, pB = 0.0;
  if constexpr (PIPE)
    normal_pair_tab(rng.draw((uint32_t)w, (uint32_t)gl, (uint32_t)a.rng_step0, 0u), pA, pB, sct, ltab);
#ifdef VB_SEP_PROF
  const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_s0 = 0, t_s1 = 0, t_s2 = 0;
#endif

  for (int s = 0; s < a.n_steps; ++s) {
    const long long i = a.step0 + s;
    const uint32_t ri = (uint32_t)(a.rng_step0 + s);
    double gA = 0.0, gB = 0.0, hA = 0.0, hB = 0.0, v = 0.0;
    double qA = 0.0, qB = 0.0;   // (kQuad: sums of x^2)
    // reparameterise one sample row of the pair, evaluate the target, accumulate;
    // PD (a.pd as a compile-time tag: the sample loop is instantiated per form, so
    // no run-time test sits in it)
    auto consume = [&](double eA, double eB, auto pdc) {
      constexpr int PD = decltype(pdc)::value;
      if constexpr (kQuad && PD == 0) {
        // isotropic Gaussian target: log p = -x^2 / 2 + const and grad = -x, so the
        // row adds x (gradient), x eps and x^2 (value, scaled and offset once per step)
        const double xA = eA * sA + muA, xB = eB * sB + muB;
        gA -= xA;
        hA = fma(-xA, eA, hA);
        qA = fma(xA, xA, qA);
        gB -= xB;
        hB = fma(-xB, eB, hB);
        qB = fma(xB, xB, qB);
        return;
      }
      double dg;
      const double xA = eA * sA + muA;
      double lpA = TGT::lp1(xA, dg);
      gA += dg;
      hA += dg * eA;
      const double xB = eB * sB + muB;
      double lpB = TGT::lp1(xB, dg);
      // -log q(x) without its per-pair constants: 1/2 eps^2 (Gaussian) or
      // (df + 1)/2 log1p(eps^2 / df) (t, df = 2 shape)
      // (the form is a run-time field: host-noise launches do not instantiate TFAM)
      if constexpr (PD == 2) {
        const double df = 2.0 * a.shape;
        lpA += 0.5 * (df + 1.0) * log1p(eA * eA / df);
        lpB += 0.5 * (df + 1.0) * log1p(eB * eB / df);
      } else if constexpr (PD == 1) {
        lpA += 0.5 * eA * eA;
        lpB += 0.5 * eB * eB;
      }
      v += fma(hbw, lpB, lpA);   // lpA + lpB, or lpA on a lane without column B
      gB += dg;
      hB += dg * eB;
    };
    // draw sample row n (host noise, or Philox normals [+ gamma for t]) and consume it
    auto sample = [&](int n, auto pdc) {
      double eA, eB;
      if constexpr (HOST) {
        const double* row = a.noise + ((long long)s * N + n) * D;
        eA = live ? row[dA] : 0.0;
        eB = hasB ? row[dB] : 0.0;
      } else {
        normal_pair_tab(rng.draw((uint32_t)w, (uint32_t)n, ri, 0u), eA, eB, sct, ltab);
        if constexpr (TFAM) {
          double GA, GB;
          gamma_pair<true>(rng, (uint32_t)w, (uint32_t)n, ri, a.shape, GA, GB, sct, ltab);
          eA = a.t_scale * eA / sqrt(GA);
          eB = a.t_scale * eB / sqrt(GB);
        }
      }
      consume(eA, eB, pdc);
    };
    // sample rows gl + k LPP: a loop with a uniform trip count over the rows every
    // lane has (scalar loop control, no exec-mask bookkeeping per row), then the
    // ragged remainder row of the lanes below N % LPP
    auto rows = [&](auto pdc) {
      int k0 = 0;
      if constexpr (PIPE) {
        // sample row gl was drawn during the previous step's update
        if (gl < N) consume(pA, pB, pdc);
        k0 = 1;
      }
      const int kfull = N / LPP;
      // (unrolled 2 or 4 times -- interleaved rows -- the launch is unchanged, 75.8 us:
      // profiles/r05/headline_unroll_rejected.log)
#pragma unroll 1
      for (int k = k0; k < kfull; ++k) sample(gl + k * LPP, pdc);
      const int kr = kfull > k0 ? kfull : k0;
      if (gl + kr * LPP < N) sample(gl + kr * LPP, pdc);
    };
    if (pdv == 0) rows(std::integral_constant<int, 0>{});
    else if (pdv == 2) rows(std::integral_constant<int, 2>{});
    else rows(std::integral_constant<int, 1>{});
    if constexpr (kQuad) {
      // the rows' log p: -1/2 sum x^2 plus the constant of each of the lane's rows
      if (pdv == 0) v = fma(hbw, fma(-0.5, qB, quad_c), fma(-0.5, qA, quad_c));
    }
    const double S = reduce4<PPW>(lane, gA, gB, hA, hB);
    // d/dmu = -mean g ; d/dlog sigma = -(1 + sigma * mean(g * eps))
    const double m = S * invN;
    const double g_own = own < 2 ? -m : -(1.0 + s_own * m);

    // value partial sum log s + mean log p over the pair; summed over lanes and
    // written for four steps at a time (vpart[step][pair])
    v3 = v2;
    v2 = v1;
    v1 = v0;
    v0 = ent ? fma(v, invN, lam_own) : v * invN;
    if ((s & 3) == 3 || s + 1 == a.n_steps) {
      const double tot = reduce4<PPW>(lane, v3, v2, v1, v0);  // owner q: step s - 3 + q
      const int st = s - 3 + own;
      if (rep && live && st >= (s & ~3)) a.vpart[(long long)st * a.n_waves + w] = tot;
    }

    if (emit_grad) {
      if (updater) a.grad[own_idx] = g_own;
      continue;
    }

    // the next step's first draw does not depend on lambda: issued here, in the
    // same basic block as the window / update / broadcast chain below, it fills
    // that chain's latency
    if constexpr (PIPE) normal_pair_tab(rng.draw((uint32_t)w, (uint32_t)gl, ri + 1u, 0u), pA, pB, sct, ltab);
    // window push (vb.py:365-370) and accum = sum of g^2 over the window
    // (vb.py:371-373).  Slots outside the window hold 0 or stale values that
    // the count mask removes.
    cnt = cnt < W ? cnt + 1 : W;
    double q;
    if constexpr (REGRING) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int sl = j * SL + sub;
        if (sl == slot) rg[j] = g_own;
        const double t = rg[j];
        acc += (sl < W) ? t * t : 0.0;
      }
      q = owner_sum<PPW>(acc);
    } else {
      if (rep) ring[slot * 4 * PPW + own] = g_own;
      int L = (cnt < W) ? 0 : (slot + 1 == W ? 0 : slot + 1);
      q = 0.0;
      for (int k = 0; k < cnt; ++k) {
        const double t = ring[L * 4 * PPW + own];
        q += t * t;
        L = (L + 1 == W) ? 0 : L + 1;
      }
    }
    // lam - lr * g / sqrt(eps + accum)   (vb.py:374)
    lam_own = lam_own - (a.lr.at(i) * g_own) * rsqrt_pos(a.eps + q);
    s_own = exp_fast(lam_own);
    muA = group_bcast<PPW, 0>(lam_own, grp);
    muB = group_bcast<PPW, 1>(lam_own, grp);
    sA = group_bcast<PPW, 2>(s_own, grp);
    sB = group_bcast<PPW, 3>(s_own, grp);
    if (i >= a.hist_start && updater) a.hist[(i - a.hist_start) * P + own_idx] = lam_own;
    slot = (slot + 1 == W) ? 0 : slot + 1;
#ifdef VB_SEP_TS
    if (lane == 0 && a.step0 == VB_SEP_TS && ((s & (s - 1)) == 0 || s + 1 == a.n_steps)) {
      const int wslot = blockIdx.x * 4 + (threadIdx.x >> 6);
      const int k = s + 1 == a.n_steps ? 13 : (s == 0 ? 0 : 1 + __builtin_ctz(s));
      if (wslot < kTsWaves) {
        g_sep_ts[wslot][k] = __builtin_amdgcn_s_memrealtime();
        g_sep_clk[wslot][k] = __builtin_amdgcn_s_memtime();
        if (s == 0) {
          g_sep_ts[wslot][14] = PPW;
          g_sep_ts[wslot][15] = t_entry;
        }
      }
    }
#endif
#ifdef VB_SEP_PROF
    if (s < 3) {
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      if (s == 0) t_s0 = t;
      else if (s == 1) t_s1 = t;
      else t_s2 = t;
    }
#endif
  }

#ifdef VB_SEP_PROF
  if (lane == 0 && a.step0 == VB_SEP_PROF) {
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    printf("SEPW %d %d %u %u %llu %llu %llu %llu %llu %llu %llu\n", PPW, w,
           __builtin_amdgcn_s_getreg(63492), __builtin_amdgcn_s_getreg(63508), t_entry, t_start,
           t_loop, t_end, t_s0, t_s1, t_s2);
  }
#endif
  if (!emit_grad && own_ok) {
    if (rep) a.lam[own_idx] = lam_own;
    if constexpr (REGRING) {
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int sl = j * SL + sub;
        if (sl < W) a.ring[(long long)sl * P + own_idx] = rg[j];
      }
    } else {
      if (rep)
        for (int k = 0; k < W; ++k) a.ring[(long long)k * P + own_idx] = ring[k * 4 * PPW + own];
    }
  }
}

// Grid: blocks [0, a.blocks2) run PPW_BIG column pairs per wave, the remaining
// blocks one pair per wave.  The split balances the work per SIMD with every
// wave resident; it affects speed only.
template <class TGT, bool TFAM, bool HOST, int PPW_BIG, bool REGRING, bool ADV = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, 256), amdgpu_waves_per_eu(3)))
void sep_kernel(SepArgs a) {
#if defined(VB_SEP_PROF) || defined(VB_SEP_TS)
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
#else
  const unsigned long long t_entry = 0;
#endif
  kernarg_warm(a);   // (every line of the arguments in the first scalar batch)
  __shared__ double s_ring[REGRING ? 1 : 4][REGRING ? 1 : 64 * 4 * PPW_BIG];
  // Box-Muller tables (vb_tables.hpp) for the in-kernel Philox draws
  __shared__ double2 s_sct[HOST ? 1 : kSinCosN];
  __shared__ double2 s_lt[HOST ? 1 : kLogN + kLogU01N];
  const int wid = threadIdx.x >> 6;
  const bool big = (int)blockIdx.x < a.blocks2;
  const int wave = blockIdx.x * 4 + wid;
  const int pair = a.pairs2 + (blockIdx.x - a.blocks2) * 4 + wid;
  SepPre<PPW_BIG> pb;
  SepPre<1> p1;
  // the lambda and register-window loads are issued before the table barrier
  // (after it, as before round 5: 5.15-5.37 vs 5.14-5.35 us/step, launch pair 79.6
  // vs 78.1 us; profiles/r05/headline_prefetch_ab_d.log)
  if (big) {
    if (wave * PPW_BIG < a.pairs2) pb = sep_pre<PPW_BIG, REGRING, ADV>(a, wave);
  } else if (pair < a.n_pairs) {
    p1 = sep_pre<1, REGRING, ADV>(a, pair);
  }
  if constexpr (!HOST) {
    load_bm_tables(s_sct, s_lt);
    __syncthreads();
  }
  double* ring = REGRING ? nullptr : &s_ring[REGRING ? 0 : wid][0];
  if (big) {
    if (wave * PPW_BIG < a.pairs2)
      sep_body<TGT, TFAM, HOST, PPW_BIG, REGRING, ADV>(a, ring, wave, s_sct, s_lt, pb, t_entry);
  } else {
    if (pair < a.n_pairs)
      sep_body<TGT, TFAM, HOST, 1, REGRING, ADV>(a, ring, pair, s_sct, s_lt, p1, t_entry);
  }
}

// values[i] = -(c0 + sum_w vpart[s][w]), fixed-order tree reduction.  One
// 1024-thread block per step; each thread issues kValU independent loads per
// round (one round covers 8 192 pairs: D = 1e4 needs one), so the block waits
// on one load latency instead of a dependent chain of n_waves / 256.
constexpr int kValThreads = 1024, kValU = 8;
__global__ __launch_bounds__(kValThreads) void sep_values_kernel(const double* vpart,
                                                                 int n_waves, double c0,
                                                                 double* values) {
  __shared__ double red[kValThreads / 64];
  const double* row = vpart + (long long)blockIdx.x * n_waves;
  double acc[kValU];
#pragma unroll
  for (int u = 0; u < kValU; ++u) acc[u] = 0.0;
  for (int base = threadIdx.x; base < n_waves; base += kValU * kValThreads) {
    double v[kValU];
#pragma unroll
    for (int u = 0; u < kValU; ++u) {
      const int w = base + u * kValThreads;
      v[u] = w < n_waves ? row[w] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kValU; ++u) acc[u] += v[u];
  }
  double t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  t = wave_sum(t);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = (red[4 * j] + red[4 * j + 1]) + (red[4 * j + 2] + red[4 * j + 3]);
    values[blockIdx.x] = -(c0 + ((r[0] + r[1]) + (r[2] + r[3])));
  }
}

// out[q][p] = mean_r hist[q][r][p]; sequential over r like numpy's axis-0 reduce.
// np.mean(hist, axis=0) per problem: numpy adds the rows in order, so each
// thread keeps that order; 64-thread blocks spread the few columns over many
// CUs and batches of 16 independent loads keep them in flight (the adds stay
// sequential).
constexpr int kRowMeanThreads = 64, kRowMeanU = 16;
__global__ __launch_bounds__(kRowMeanThreads) void row_mean_kernel(const double* hist, long long rows,
                                                                   long long P, long long nprob,
                                                                   double* out) {
  const long long idx = (long long)blockIdx.x * kRowMeanThreads + threadIdx.x;
  if (idx >= P * nprob) return;
  const long long q = idx / P, p = idx % P;
  const double* h = hist + q * rows * P + p;
  double acc = 0.0;
  long long r = 0;
  for (; r + kRowMeanU <= rows; r += kRowMeanU) {
    double v[kRowMeanU];
#pragma unroll
    for (int u = 0; u < kRowMeanU; ++u) v[u] = h[(r + u) * P];
#pragma unroll
    for (int u = 0; u < kRowMeanU; ++u) acc += v[u];
  }
  for (; r < rows; ++r) acc += h[r * P];
  out[idx] = acc / (double)rows;
}

// -------------------------------------------------------------------------
// block-per-problem kernel (any target, D <= DMAX), KLVI and CHIVI
// -------------------------------------------------------------------------
template <class TGT>
using RowOf = std::conditional_t<TGT::kSeparable, SepRow<TGT>, TGT>;

// Wave-level reduce-scatter of K per-lane values: two permlane swap levels fold
// four values into each register (halves, then rows), a 4-step DPP row sum
// finishes them, and lane 0 of each row writes its value's wave total to
// out[k].  ~3x fewer instructions than K full-wave sums.
__device__ __forceinline__ double swap32_pair(double a, double b) {
  const auto l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a),
                                                  (unsigned)__double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a),
                                                  (unsigned)__double2hiint(b), false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}

__device__ __forceinline__ double swap16_pair(double a, double b) {
  const auto l = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a),
                                                  (unsigned)__double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a),
                                                  (unsigned)__double2hiint(b), false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}

template <int K>
__device__ __forceinline__ void wave_reduce_scatter(const double (&v)[K], double* out) {
  constexpr int H1 = (K + 1) / 2, H2 = (H1 + 1) / 2;
  double r1[H1], r2[H2];
#pragma unroll
  for (int i = 0; i < H1; ++i) r1[i] = swap32_pair(v[i], i + H1 < K ? v[i + H1] : 0.0);
#pragma unroll
  for (int j = 0; j < H2; ++j) {
    double t = swap16_pair(r1[j], j + H2 < H1 ? r1[j + H2] : 0.0);
    t += dpp_f64<0xB1>(t);   // quad_perm [1,0,3,2]
    t += dpp_f64<0x4E>(t);   // quad_perm [2,3,0,1]
    t += dpp_f64<0x141>(t);  // row_half_mirror
    t += dpp_f64<0x140>(t);  // row_mirror
    r2[j] = t;
  }
  const int lane = threadIdx.x & 63, q = lane >> 4;
  if ((lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < H2; ++j) {
      const int i = j + (q & 1) * H2;  // row q of register j holds v[i + (q >> 1) * H1]
      const int k = i + (q >> 1) * H1;
      if (i < H1 && k < K) out[k] = r2[j];
    }
  }
}

// Split rows: the same reduce-scatter over the lanes of one parity (lane h of
// every pair holds register j for output index map(j, h)): the in-row steps are
// lane ^ 2, row_ror 4 and row_ror 8 (parity preserving), and lanes 0 / 1 of each
// row write the even / odd totals.  Register j < DH is coordinate h DH + j's
// gradient sum, DH <= j < 2 DH the (g e) sum of coordinate h DH + j - DH, j = 2 DH
// the log p / weight sum (even lanes only; odd lanes hold zero).
template <int KH, int DH, int DMAX>
__device__ __forceinline__ void wave_reduce_scatter_pair(const double (&v)[KH], double* out) {
  constexpr int H1 = (KH + 1) / 2, H2 = (H1 + 1) / 2;
  double r1[H1], r2[H2];
#pragma unroll
  for (int i = 0; i < H1; ++i) r1[i] = swap32_pair(v[i], i + H1 < KH ? v[i + H1] : 0.0);
#pragma unroll
  for (int j = 0; j < H2; ++j) {
    double t = swap16_pair(r1[j], j + H2 < H1 ? r1[j + H2] : 0.0);
    t += dpp_f64<0x4E>(t);   // quad_perm [2,3,0,1]: lane ^ 2
    t += dpp_f64<0x124>(t);  // row_ror:4
    t += dpp_f64<0x128>(t);  // row_ror:8
    r2[j] = t;
  }
  const int lane = threadIdx.x & 63, q = lane >> 4, pos = lane & 15;
  if (pos < 2) {
    const int h = pos;
#pragma unroll
    for (int j = 0; j < H2; ++j) {
      const int i = j + (q & 1) * H2;
      const int k = i + (q >> 1) * H1;
      if (i < H1 && k < KH) {
        const int idx = k < DH ? h * DH + k : k < 2 * DH ? DMAX + h * DH + (k - DH) : (h == 0 ? 2 * DMAX : -1);
        if (idx >= 0) out[idx] = r2[j];
      }
    }
  }
}

// Philox mode runs the block as row waves (reparameterise, target, accumulate:
// one thread per sample) and draw waves (normal pair [+ gamma pair] and the
// pair's log q partial per (sample, pair) item, into LDS).  When one step's
// draws fit half of the draw buffer the two roles overlap: draw waves produce
// step s+1 into the other half while row waves consume step s.  Otherwise
// (large N) all waves draw a chunk, then the row waves consume it.
constexpr int kBlockMaxThreads = 512;
constexpr int kBlockDrawLds = 4096;  // doubles of LDS for the draw records
constexpr int kBlockMaxRowWaves = 4;

// Device-noise path: a copy wave stages step s + 2's noise rows (and log q
// partials) into a 3-slot LDS ring with LDS-DMA loads while the row waves work
// on step s, so no step waits on an HBM round trip for its rows.  Slot layout:
// [N D noise | N lq], each part rounded up to whole 128-double DMA instructions.
constexpr int kBlockPfLds = 4608;    // doubles of LDS for the 3-slot ring (36 KB)
constexpr int kPfUnit = 128;         // doubles per wave-wide 16-byte DMA instruction

// Row reads of the copy wave's ring: DMAX ds_read_b64 at immediate offsets from
// one row address [+ the row's log q partial], and the lgkmcnt(0) wait, in ONE
// asm statement.  Every destination is an output of the statement that also
// waits, so the compiler cannot copy or spill a register whose LDS load is still
// in flight (the hardware has no interlock for that).  Generated per DMAX
// instance (2, 4, 10, 16) with and without the log q read.
template <int DMAX> struct LdsRowWait;
template <> struct LdsRowWait<2> {
  static __device__ __forceinline__ void run(unsigned a, unsigned q, bool lq, double (&e)[2],
                                               double& tl) {
    if (lq) {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[t], %[q]\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [t] "=&v"(tl)
                   : [a] "v"(a), [q] "v"(q)
                   : "memory");
    } else {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1])
                   : [a] "v"(a)
                   : "memory");
    }
  }
};
template <> struct LdsRowWait<4> {
  static __device__ __forceinline__ void run(unsigned a, unsigned q, bool lq, double (&e)[4],
                                               double& tl) {
    if (lq) {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "ds_read_b64 %[t], %[q]\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3]), [t] "=&v"(tl)
                   : [a] "v"(a), [q] "v"(q)
                   : "memory");
    } else {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3])
                   : [a] "v"(a)
                   : "memory");
    }
  }
};
template <> struct LdsRowWait<10> {
  static __device__ __forceinline__ void run(unsigned a, unsigned q, bool lq, double (&e)[10],
                                               double& tl) {
    if (lq) {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "ds_read_b64 %[e4], %[a] offset:32\n"
                   "ds_read_b64 %[e5], %[a] offset:40\n"
                   "ds_read_b64 %[e6], %[a] offset:48\n"
                   "ds_read_b64 %[e7], %[a] offset:56\n"
                   "ds_read_b64 %[e8], %[a] offset:64\n"
                   "ds_read_b64 %[e9], %[a] offset:72\n"
                   "ds_read_b64 %[t], %[q]\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3]), [e4] "=&v"(e[4]), [e5] "=&v"(e[5]), [e6] "=&v"(e[6]), [e7] "=&v"(e[7]), [e8] "=&v"(e[8]), [e9] "=&v"(e[9]), [t] "=&v"(tl)
                   : [a] "v"(a), [q] "v"(q)
                   : "memory");
    } else {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "ds_read_b64 %[e4], %[a] offset:32\n"
                   "ds_read_b64 %[e5], %[a] offset:40\n"
                   "ds_read_b64 %[e6], %[a] offset:48\n"
                   "ds_read_b64 %[e7], %[a] offset:56\n"
                   "ds_read_b64 %[e8], %[a] offset:64\n"
                   "ds_read_b64 %[e9], %[a] offset:72\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3]), [e4] "=&v"(e[4]), [e5] "=&v"(e[5]), [e6] "=&v"(e[6]), [e7] "=&v"(e[7]), [e8] "=&v"(e[8]), [e9] "=&v"(e[9])
                   : [a] "v"(a)
                   : "memory");
    }
  }
};
template <> struct LdsRowWait<16> {
  static __device__ __forceinline__ void run(unsigned a, unsigned q, bool lq, double (&e)[16],
                                               double& tl) {
    if (lq) {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "ds_read_b64 %[e4], %[a] offset:32\n"
                   "ds_read_b64 %[e5], %[a] offset:40\n"
                   "ds_read_b64 %[e6], %[a] offset:48\n"
                   "ds_read_b64 %[e7], %[a] offset:56\n"
                   "ds_read_b64 %[e8], %[a] offset:64\n"
                   "ds_read_b64 %[e9], %[a] offset:72\n"
                   "ds_read_b64 %[e10], %[a] offset:80\n"
                   "ds_read_b64 %[e11], %[a] offset:88\n"
                   "ds_read_b64 %[e12], %[a] offset:96\n"
                   "ds_read_b64 %[e13], %[a] offset:104\n"
                   "ds_read_b64 %[e14], %[a] offset:112\n"
                   "ds_read_b64 %[e15], %[a] offset:120\n"
                   "ds_read_b64 %[t], %[q]\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3]), [e4] "=&v"(e[4]), [e5] "=&v"(e[5]), [e6] "=&v"(e[6]), [e7] "=&v"(e[7]), [e8] "=&v"(e[8]), [e9] "=&v"(e[9]), [e10] "=&v"(e[10]), [e11] "=&v"(e[11]), [e12] "=&v"(e[12]), [e13] "=&v"(e[13]), [e14] "=&v"(e[14]), [e15] "=&v"(e[15]), [t] "=&v"(tl)
                   : [a] "v"(a), [q] "v"(q)
                   : "memory");
    } else {
      asm volatile("ds_read_b64 %[e0], %[a] offset:0\n"
                   "ds_read_b64 %[e1], %[a] offset:8\n"
                   "ds_read_b64 %[e2], %[a] offset:16\n"
                   "ds_read_b64 %[e3], %[a] offset:24\n"
                   "ds_read_b64 %[e4], %[a] offset:32\n"
                   "ds_read_b64 %[e5], %[a] offset:40\n"
                   "ds_read_b64 %[e6], %[a] offset:48\n"
                   "ds_read_b64 %[e7], %[a] offset:56\n"
                   "ds_read_b64 %[e8], %[a] offset:64\n"
                   "ds_read_b64 %[e9], %[a] offset:72\n"
                   "ds_read_b64 %[e10], %[a] offset:80\n"
                   "ds_read_b64 %[e11], %[a] offset:88\n"
                   "ds_read_b64 %[e12], %[a] offset:96\n"
                   "ds_read_b64 %[e13], %[a] offset:104\n"
                   "ds_read_b64 %[e14], %[a] offset:112\n"
                   "ds_read_b64 %[e15], %[a] offset:120\n"
                   "s_waitcnt lgkmcnt(0)"
                   : [e0] "=&v"(e[0]), [e1] "=&v"(e[1]), [e2] "=&v"(e[2]), [e3] "=&v"(e[3]), [e4] "=&v"(e[4]), [e5] "=&v"(e[5]), [e6] "=&v"(e[6]), [e7] "=&v"(e[7]), [e8] "=&v"(e[8]), [e9] "=&v"(e[9]), [e10] "=&v"(e[10]), [e11] "=&v"(e[11]), [e12] "=&v"(e[12]), [e13] "=&v"(e[13]), [e14] "=&v"(e[14]), [e15] "=&v"(e[15])
                   : [a] "v"(a)
                   : "memory");
    }
  }
};

struct BlockLayout {
  int nt, rw, pipe, rec;  // threads, row waves, overlapped draws, doubles per sample record
  int pf;                 // device noise prefetched by a copy wave (the last wave)
  int pf_lq, pf_slot;     // doubles offset of the lq part in a slot, doubles per slot
  int split;              // two row lanes per sample, each with half of the coordinates
};

// Split rows (copy-wave layout, 2 <= D <= 10, N <= 128): lanes 2j and 2j + 1 of a
// row wave share sample j; lane h takes coordinates [h DH, h DH + DH), DH =
// ceil(DMAX / 2), and the pair exchanges its cross-coordinate sums (log p, the
// shared-coordinate gradients) with one DPP swap.  A step is a dependent chain of
// one wave's instructions (one wave per SIMD), so halving each lane's
// per-coordinate work and spreading the samples over up to 4 row waves (all four
// SIMDs) shortens it; the copy wave shares a SIMD.
constexpr int kBlockSplitMaxD = 10;
constexpr int kBlockQpreMaxW = 16;   // windows the copy wave pre-sums (block_kernel)

__host__ __device__ inline int pf_round(int n) { return (n + kPfUnit - 1) / kPfUnit * kPfUnit; }

__host__ __device__ inline BlockLayout block_layout(int N, int D, bool host, bool need_lq,
                                                   int pf_ok = 0) {
  const int NP = (D + 1) / 2;
  const int rw = std::min(kBlockMaxRowWaves, std::max(1, (N + 63) / 64));
  BlockLayout L{};
  L.rw = rw;
  L.rec = 2 * NP + (need_lq ? NP : 0);
  if (host) {
    L.nt = 64 * rw;
    L.pipe = 0;
    L.pf_lq = pf_round(N * D);
    L.pf_slot = L.pf_lq + (need_lq ? pf_round(N) : 0);
    // at most 3 row waves + the copy wave: the PF instances launch with <= 256
    // threads (one wave per SIMD), so their registers may reach the whole file
    L.pf = pf_ok && rw <= 3 && 3 * L.pf_slot <= kBlockPfLds;
    if (pf_ok == 2 && D >= 2 && D <= kBlockSplitMaxD && 2 * N <= 64 * kBlockMaxRowWaves &&
        3 * L.pf_slot <= kBlockPfLds) {
      L.split = 1;
      L.pf = 1;
      L.rw = (2 * N + 63) / 64;
      L.nt = 64 * L.rw;
    }
    if (L.pf) L.nt += 64;
    return L;
  }
  const long long iw = ((long long)N * NP + 63) / 64;  // waves of draw items
  const int maxw = kBlockMaxThreads / 64;
  if ((long long)N * L.rec <= kBlockDrawLds / 2) {
    L.pipe = 1;
    L.nt = 64 * (rw + (int)std::min<long long>(maxw - rw, std::max<long long>(1, iw)));
  } else {
    L.pipe = 0;
    L.nt = 64 * (int)std::min<long long>(maxw, std::max<long long>(rw, iw));
  }
  return L;
}

template <class TGT, bool TFAM, bool HOST, int DMAX, bool PF = false, bool SPLIT = false, int HOT = 0>
// device-noise (HOST) instances launch <= 256 threads (<= 4 row waves, or <= 3 and the
// copy wave): one wave per SIMD, so their registers may use the whole file instead of
// spilling at the 256-VGPR cap a 512-thread bound implies (the DMAX = 16 instances).
// Split-row instances (DMAX <= 10) launch up to 4 row waves + the copy wave.
__global__ __launch_bounds__(HOST ? (SPLIT ? 320 : 256) : kBlockMaxThreads) void block_kernel(BlockArgs a) {
  static_assert(!SPLIT || (HOST && PF && DMAX <= kBlockSplitMaxD), "split rows: copy-wave layout");
  // HOT (split-row instances only): the objective / optimiser flags of the benchmark
  // configurations as compile-time constants -- 1 KLVI + windowed adagrad, 2 CHIVI +
  // windowed adagrad, no emitted gradient, no sampled log q -- so their runs carry no
  // branch, mask or reload for the other modes (0: the flags as passed)
  static_assert(HOT == 0 || SPLIT, "compile-time modes for the split-row instances");
  const bool k_chivi = HOT == 2 ? true : (HOT == 1 ? false : (bool)a.chivi);
  const bool k_pd = HOT ? false : (bool)a.pd;
  const int k_opt = HOT ? 0 : a.opt;
  const bool k_emit = HOT ? false : (bool)a.emit_grad;
  constexpr int K = 2 * DMAX + 2;   // G[DMAX], H[DMAX], V/S, spare
  constexpr int DH = (DMAX + 1) / 2, KH = 2 * DH + 1;   // split rows: per-lane half
  constexpr int WMAX = 64;
  __shared__ double s_lam[2 * DMAX];
  __shared__ double s_sg[DMAX];     // exp(log sigma) of the current lam
  __shared__ double s_ring[WMAX * 2 * DMAX];
  __shared__ double s_red[kBlockMaxRowWaves][K];
  __shared__ double s_max[kBlockMaxRowWaves];
  __shared__ double2 s_sct[HOST ? 1 : kSinCosN];
  __shared__ double2 s_lt[HOST ? 1 : kLogN + kLogU01N];
  __shared__ double s_e[HOST ? 1 : kBlockDrawLds + DMAX];  // + slack for the row loads
  __shared__ __attribute__((aligned(16))) double s_pf[HOST && PF ? kBlockPfLds + kBlockDMax : 1];
  __shared__ double s_qold[HOST && PF ? 2 * DMAX : 1];   // window sums without the newest slot
  // KLVI (qnext): the window sums of step s without its two newest slots, by step parity
  __shared__ double s_qpre[2][HOST && PF ? 2 * DMAX : 1];
  __shared__ double s_sl;   // copy-wave layout: sum_d log sigma_d of the step's lam
  if constexpr (!HOST) load_bm_tables(s_sct, s_lt);

  using Row = RowOf<TGT>;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int NT = blockDim.x;
  const int prob = blockIdx.x;
  const int D = a.D, N = a.N, W = a.W, P = a.P;
  const bool need_lq = k_chivi || k_pd;
  const BlockLayout L = block_layout(N, D, HOST, need_lq, (HOST && PF) ? a.pf : 0);
  const int RW = L.rw, RT = 64 * RW, R = L.rec;
  const bool row_wave = wid < RW;
  // PF instances are launched exactly when the layout has the copy wave (block_dispatch_dm)
  constexpr bool kPF = HOST && PF;
  const bool copy_wave = kPF && wid == RW;   // the last wave (block_layout)
  const int NTw = kPF ? NT - 64 : NT;        // threads of the row / draw waves
  const int val_tid = NTw > 64 ? NTw - 64 : 0;  // value on another wave than the update
  // (the CHIVI HOT instance is launched only with the pre-drawn log q partials:
  // block_dispatch_dm)
  const bool pre_lq = HOST && (HOT == 2 ? true : a.noise_lq != nullptr);
  // copy wave: noise rows (and log q partials) of step s -> ring slot s % 3, as
  // wave-wide 16-byte LDS-DMA loads (4-byte ones when a source is not 16-byte
  // aligned); lanes past the end re-read the first element into the slot's slack
  auto pf_copy = [&](const double* src, double* dst, int nd) __attribute__((always_inline)) {
    if ((((uintptr_t)src) & 15) == 0 && (nd & 1) == 0) {
      for (int o = 0; o < nd; o += kPfUnit) {
        const int e = o + 2 * lane;
        __builtin_amdgcn_global_load_lds((const void*)(src + (e < nd ? e : 0)), (void*)(dst + o),
                                         16, 0, 0);
      }
    } else {
      const int* s4 = reinterpret_cast<const int*>(src);
      int* d4 = reinterpret_cast<int*>(dst);
      for (int o = 0; o < 2 * nd; o += 64) {
        const int e = o + lane;
        __builtin_amdgcn_global_load_lds((const void*)(s4 + (e < 2 * nd ? e : 0)), (void*)(d4 + o),
                                         4, 0, 0);
      }
    }
  };
  auto pf_issue = [&](int s) __attribute__((always_inline)) {
    if constexpr (kPF) {
      const long long rix = ((long long)prob * a.n_steps + s) * N;
      double* slot_p = s_pf + (s % 3) * L.pf_slot;
      pf_copy(a.noise + rix * D, slot_p, N * D);
      if (need_lq && pre_lq) pf_copy(a.noise_lq + rix, slot_p + L.pf_lq, N);
    }
  };
  const double dN = (double)N;
  // 1 / N once per launch: the update multiplies (exact for a power-of-two N, within
  // an ulp otherwise) instead of dividing on its serial chain
  const double inv_dN = 1.0 / dN;
  // adagrad window sums: the copy wave adds up the older W - 1 slots of every
  // parameter while the rows run (same order, oldest first), so the update adds
  // only the newest square (the same bits as the whole loop)
  // (the CHIVI HOT instance is launched only for windows the copy wave pre-sums:
  // block_dispatch_dm; the general window loop then drops out of its code -- config 2
  // 2.06 -> 1.81 us/step with the pre-drawn log q below; the same for the KLVI instance
  // cost config 5's fit 7.8 -> 8.05 ms, profiles/r06/hot_compile_time_facts_ab.log)
  const bool qpre = HOT == 2 ? true : (kPF && k_opt == 0 && !k_emit && W >= 1 && W <= kBlockQpreMaxW);
  // The copy wave sums step s + 1's window (but its newest slot) after step s's
  // reduction barrier, beside the update, instead of before that barrier, which it held
  // (KLVI, profiles/r05/copy_wave_ts.log; CHIVI from round 6: its sums after the block-
  // max barrier made the rows wait ~575 cycles at the reduction barrier,
  // profiles/r06/block_ts.log); the update adds the previous gradient's square (gprev)
  // and its own -- the same additions in the same order
  const bool qnext = qpre && W >= 2;
  double* lam_g = a.lam + (long long)prob * P;
  double* ring_g = a.ring ? a.ring + (long long)prob * W * P : nullptr;

  for (int p = tid; p < P; p += NT) s_lam[p] = lam_g[p];
  if (!k_emit)
    for (int q = tid; q < W * P; q += NT) s_ring[q] = ring_g[q];
  for (int d = tid; d < D; d += NT) s_sg[d] = exp_fast(lam_g[D + d]);
  // the reduction rows of absent row waves hold zeros (never written after this), so
  // every column sum adds all kBlockMaxRowWaves rows: no select on the update's chain
  for (int q = RW * K + tid; q < kBlockMaxRowWaves * K; q += NT) (&s_red[0][0])[q] = 0.0;

  const Rng rng{a.k0, a.k1, (uint32_t)(a.stream + (uint32_t)prob * a.stream_stride)};
  const double c0 = TFAM ? 0.0 : 0.5 * D * (1.0 + kLog2Pi);
  const int NP = (D + 1) / 2;
  const double lq_half = 0.5 * (a.df + 1.0);
  const double inv_df = 1.0 / a.df;

  // one (sample, pair) draw item: e pair [+ log q partial of the pair, sans -log sigma].
  // Always inlined: the t instances once kept it out of line, where `buf` (an LDS
  // array) became a generic pointer and its two-double record stores were merged
  // into flat 16-byte stores at 8-byte-aligned LDS addresses (odd record lengths:
  // CHIVI's 3 NP, and the s_e base itself is only 8-byte aligned) -- the memory
  // aperture violation of the in-kernel t sampler.  Inlined, the
  // stores are ds_write_b64 / ds_write2_b64 on the LDS array.
  auto draw_item = [&](int it0, int it_step, int n_items, int nbase, long long ri,
                       double* buf) __attribute__((always_inline)) {
    for (int it = it0; it < n_items; it += it_step) {
      const int nl = it / NP, j = it - nl * NP;
      const uint32_t n = (uint32_t)(nbase + nl);
      double ea, eb;
      normal_pair_tab(rng.draw((uint32_t)j, n, (uint32_t)ri, 0u), ea, eb, s_sct, s_lt);
      if constexpr (TFAM) {
        double ga, gb;
        gamma_pair<true>(rng, (uint32_t)j, n, (uint32_t)ri, a.shape, ga, gb, s_sct, s_lt);
        // t = sqrt(df / 2) z / sqrt(G): a refined rsqrt instead of sqrt + divide
        ea = a.t_scale * ea * rsqrt_pos(ga);
        eb = a.t_scale * eb * rsqrt_pos(gb);
      }
      double* rec = buf + nl * R;
      rec[2 * j] = ea;
      rec[2 * j + 1] = eb;
      if (need_lq) {
        const bool hasb = 2 * j + 1 < D;
        double lqp;
        if constexpr (TFAM) {
#ifdef VB_NO_LQ_TAB
          lqp = a.t_const - log1p(ea * ea * inv_df) * lq_half;
          if (hasb) lqp += a.t_const - log1p(eb * eb * inv_df) * lq_half;
#else
          lqp = a.t_const - log1p_pos_tab(ea * ea * inv_df, s_lt) * lq_half;
          if (hasb) lqp += a.t_const - log1p_pos_tab(eb * eb * inv_df, s_lt) * lq_half;
#endif
        } else {
          lqp = -0.5 * ea * ea - 0.5 * kLog2Pi;
          if (hasb) lqp += -0.5 * eb * eb - 0.5 * kLog2Pi;
        }
        rec[2 * NP + j] = lqp;
      }
    }
  };

  if (copy_wave && a.n_steps > 0) {
    pf_issue(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.n_steps > 1) pf_issue(1);
  }
  __syncthreads();  // Box-Muller tables, lam, ring and sigma (and step 0's rows) are in LDS
  if constexpr (!HOST) {
    if (L.pipe && a.n_steps > 0) {
      draw_item(tid, NT, N * NP, 0, a.rng_step0, s_e);
      __syncthreads();
    }
  }

#ifdef VB_BLOCK_PROF
  unsigned long long ph[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long tw0 = wall_clock64(), tc0 = clock64(), tp = clock64();
#define VB_PH(k) do { __builtin_amdgcn_s_waitcnt(0xC07F); const unsigned long long t_ = clock64(); ph[k] += t_ - tp; tp = t_; } while (0)
#else
#define VB_PH(k) do {} while (0)
#endif
#ifdef VB_BLOCK_TS
  // barrier-exit timestamps (no waits): thread 0 of problem 0 -- a row thread and
  // the update thread of parameter 0 -- accumulates the clock64 cycles between
  // marks A step start, B rows done, C CHIVI max barrier left, D reduce-scatter
  // issued, E reduction barrier left, F own update done, G end barrier left
  unsigned long long bt[6] = {0, 0, 0, 0, 0, 0}, tb = clock64();
  const unsigned long long tb0 = tb;
#define VB_BT(k) do { const unsigned long long t_ = clock64(); bt[k] += t_ - tb; tb = t_; } while (0)
#else
#define VB_BT(k) do {} while (0)
#endif

  int slot = W > 0 ? (int)(a.step0 % W) : 0;  // window ring slot of step i (i % W)
  double gprev = 0.0;   // (qnext) the update thread's gradient of the previous step
  // split rows: the target's per-lane constants, made once (Row::lane_const)
  double lk[2 * DH] = {};
  if constexpr (SPLIT) Row::template lane_const<DH>(tid & 1, lk);
  // One step.  RO = 0: every wave runs the whole step (host noise, chunked
  // draws); with overlapped draws the row waves (RO = 1) and the draw waves
  // (RO = 2) run their own copies of the step loop — same barriers, disjoint
  // work — so neither role's registers are held across the other's code.
  auto step = [&](int s, auto role_tag) {
    constexpr int RO = decltype(role_tag)::value;
    const bool rows = RO == 1 || (RO == 0 && row_wave);
    const long long i = a.step0 + s;
    const long long ri = a.rng_step0 + s;
    // CHIVI: the update's step size and (qnext) the window's pre-sum of this step, formed
    // / read at the step's start by the update threads: the schedule's division and an
    // LDS round trip had sat on the update's serial chain after the reduction barrier
    // (round-6 ISA of the config-2 instance; config 2 2.33 -> 2.25 us/step with the
    // column reads below).  KLVI keeps them after the barrier: its rows are short, and
    // the extra work at the step's start made wave 0 late (config 1 1.00 -> 1.11,
    // profiles/r06/block_update_chain_ab.log).  s_qpre[s & 1] was written during step
    // s - 1, before its end barrier.
    double lr_i = 0.0, qo_pre = 0.0;
    if (k_chivi && RO != 2 && tid < P && !k_emit && k_opt == 0) {
      lr_i = a.lr.at(i);
      if (qnext && s > 0) qo_pre = s_qpre[s & 1][tid];
    }
    // sum_d log sigma_d of the pre-update lam: only the value needs it (log q
    // enters the rows without it: a per-step constant that cancels in the CHIVI
    // weights, added back to the value).  The copy wave computes it off the rows'
    // chain (s_sl); other layouts here, in the same order.
    double sl = 0.0;
    if constexpr (!kPF) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const double l = s_lam[D + d];
        sl += d < D ? l : 0.0;
      }
    }
    double acc[K];   // (unused by split rows: the compiler drops it)
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    double acch[KH];   // split rows: this lane's half (wave_reduce_scatter_pair; else unused)
#pragma unroll
    for (int k = 0; k < KH; ++k) acch[k] = 0.0;
    double mloc = -INFINITY;  // CHIVI: running max of this thread's log weights
    // overlapped draws: items [0, cut_a) of step s + 1 are drawn while the rows
    // consume step s, the rest during the update (see below)
#ifdef VB_NO_DRAW_SPLIT
    const int cut_a = N * NP;
#else
    const int d_lanes = NT - RT, d_rounds = (N * NP + d_lanes - 1) / max(d_lanes, 1);
    const int cut_a = d_rounds >= 2 ? (d_rounds - 1) * d_lanes : N * NP;
#endif
    VB_PH(0);

    auto row_of = [&](const double* e, double lqs) {
      double x[DMAX], g[DMAX];
      // mu and sigma straight from LDS (broadcast reads): one sample per thread
      // per step, so holding them in registers across the step buys nothing
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const double m = s_lam[d], sgd = s_sg[d];
        x[d] = d < D ? e[d] * sgd + m : 0.0;
        g[d] = 0.0;
      }
      double lp = Row::template row<DMAX>(x, g, D);
      // log q(x; lam) + sum_d log sigma_d (mvn.logpdf / t.logpdf with all
      // constants, z = eps): the sigma term is added back in the value
      const double lq = lqs;
      if (k_pd) lp -= lq;
      if (!k_chivi) {
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          acc[d] += g[d];
          acc[DMAX + d] += g[d] * e[d];
        }
        acc[2 * DMAX] += lp;
      } else {
        const double lw = lp - lq;
        if (mloc == -INFINITY && lw > -INFINITY && lw < INFINITY) {
          // a thread's first sample (the only one when N <= the row threads): the
          // general path below rescales zero accumulators by 0 and weights the
          // sample by exp(0) = 1 -- the same bits without the exp and the K-wide
          // rescale
          mloc = lw;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            acc[d] += g[d];
            acc[DMAX + d] += g[d] * e[d];
          }
          acc[2 * DMAX] += 1.0;
          return;
        }
        if (lw > mloc) {
          const double f = (mloc == -INFINITY) ? 0.0 : exp_fast(a.alpha * (mloc - lw));
#pragma unroll
          for (int k = 0; k <= 2 * DMAX; ++k) acc[k] *= f;
          mloc = lw;
        }
        const double wgt = exp_fast(a.alpha * (lw - mloc));
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          acc[d] += wgt * g[d];
          acc[DMAX + d] += wgt * (g[d] * e[d]);
        }
        acc[2 * DMAX] += wgt;
      }
    };

    // split rows: lane h of the pair (eh = its half of the noise, e = the whole
    // row for the shared coordinates 0 and 1); log p summed over the pair
    // (mu, sigma of the lane's coordinates and of coordinates 0 / 1: read by the
    // split-row block below before the row's noise, so the noise reads' wait covers
    // them -- one LDS round trip per row instead of one per coordinate read under
    // its own per-lane d < D test)
    double mk[DH], sk[DH], m01[2], s01[2];
    auto row_half_of = [&](const double* eh, const double* e, double lqs, int h) {
      double xh[DH], gh[DH];
#pragma unroll
      for (int k = 0; k < DH; ++k) {
        const int d = h * DH + k;
        xh[k] = d < D ? eh[k] * sk[k] + mk[k] : 0.0;
        gh[k] = 0.0;
      }
      const double x0 = e[0] * s01[0] + m01[0], x1 = e[1] * s01[1] + m01[1];
      double lp = Row::template row_half<DMAX, DH>(xh, gh, h, D, x0, x1, lk);
      lp += dpp_f64<0xB1>(lp);   // the pair's total (the same sum in both lanes)
      const double lq = lqs;   // (+ sum_d log sigma_d, as row_of)
      if (k_pd) lp -= lq;
      const double own = h == 0 ? 1.0 : 0.0;   // the log p / weight slot: lane 0 only
      if (!k_chivi) {
#pragma unroll
        for (int k = 0; k < DH; ++k) {
          acch[k] += gh[k];
          acch[DH + k] += gh[k] * eh[k];
        }
        acch[2 * DH] += own * lp;
      } else {
        const double lw = lp - lq;
        if (mloc == -INFINITY && lw > -INFINITY && lw < INFINITY) {
          mloc = lw;
#pragma unroll
          for (int k = 0; k < DH; ++k) {
            acch[k] += gh[k];
            acch[DH + k] += gh[k] * eh[k];
          }
          acch[2 * DH] += own;
          return;
        }
        if (lw > mloc) {
          const double f = (mloc == -INFINITY) ? 0.0 : exp_fast(a.alpha * (mloc - lw));
#pragma unroll
          for (int k = 0; k < KH; ++k) acch[k] *= f;
          mloc = lw;
        }
        const double wgt = exp_fast(a.alpha * (lw - mloc));
#pragma unroll
        for (int k = 0; k < DH; ++k) {
          acch[k] += wgt * gh[k];
          acch[DH + k] += wgt * (gh[k] * eh[k]);
        }
        acch[2 * DH] += own * wgt;
      }
    };

    if constexpr (SPLIT) {
      if (rows) {
        typedef __attribute__((address_space(3))) double lds_f64;
        const double* buf = s_pf + (s % 3) * L.pf_slot;
        const unsigned base = (unsigned)(uintptr_t)((const lds_f64*)buf);
        const int h = tid & 1;
        // this step's mu and sigma (clamped indices: every lane reads, no masked
        // block), issued before the first row's noise reads and waited for with them
#pragma unroll
        for (int k = 0; k < DH; ++k) {
          const int d = h * DH + k, dc = d < D ? d : 0;
          mk[k] = s_lam[dc];
          sk[k] = s_sg[dc];
        }
        m01[0] = s_lam[0];
        m01[1] = s_lam[1];
        s01[0] = s_sg[0];
        s01[1] = s_sg[1];
        // pairs are active together (n is the same for both lanes): the DPP swaps
        // inside row_half_of see their partner.  One sample per lane pair at most
        // (block_layout's split rows have RT >= 2 N): for DMAX >= 4 without the loop --
        // config 2 2.14 -> 2.05 us/step, config 5's fit 8.55 -> 8.0 ms; the DMAX = 2
        // instance (config 1) measured 1.00 -> 1.02 without it and keeps the loop
        // (profiles/r06/split_rows_no_loop_ab.log)
        auto split_row = [&](int n) __attribute__((always_inline)) {
          double e[DMAX];
          double tl = 0.0;
          LdsRowWait<DMAX>::run(base + 8u * (unsigned)(n * D), base + 8u * (unsigned)(L.pf_lq + n),
                                need_lq && pre_lq, e, tl);
          double eh[DH];
          double lqs = 0.0;
#pragma unroll
          for (int k = 0; k < DH; ++k) {
            const double hi = DH + k < DMAX ? e[DH + k] : 0.0;
            const double v = h ? hi : e[k];
            eh[k] = h * DH + k < D ? v : 0.0;
            if (need_lq && !pre_lq && h * DH + k < D) {
              if constexpr (TFAM)
                lqs += a.t_const - log1p(eh[k] * eh[k] / a.df) * lq_half;
              else
                lqs += -0.5 * eh[k] * eh[k] - 0.5 * kLog2Pi;
            }
          }
          if (need_lq && !pre_lq) lqs += dpp_f64<0xB1>(lqs);
          if (need_lq && pre_lq) lqs = tl;
          row_half_of(eh, e, lqs, h);
        };
        if constexpr (DMAX >= 4) {
          const int n = tid >> 1;
          if (n < N) split_row(n);
        } else {
          for (int n = tid >> 1; n < N; n += RT >> 1) split_row(n);
        }
      }
    } else if constexpr (kPF) {
      if (rows) {
        typedef __attribute__((address_space(3))) double lds_f64;
        const double* buf = s_pf + (s % 3) * L.pf_slot;
        const unsigned base = (unsigned)(uintptr_t)((const lds_f64*)buf);
        for (int n = tid; n < N; n += RT) {
          double e[DMAX];
          double lqs = 0.0;
          // LDS reads as inline asm: the compiler cannot tell these slots from
          // the copy wave's DMA targets and would wait vmcnt(0) (this wave's
          // own outstanding stores) before each; the barriers order them.  One
          // row address + immediate offsets (d >= D reads the next row or the
          // ring's slack, discarded by the select below)
          double tl = 0.0;
          LdsRowWait<DMAX>::run(base + 8u * (unsigned)(n * D), base + 8u * (unsigned)(L.pf_lq + n),
                                need_lq && pre_lq, e, tl);
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            e[d] = d < D ? e[d] : 0.0;
            if (need_lq && !pre_lq && d < D) {
              if constexpr (TFAM)
                lqs += a.t_const - log1p(e[d] * e[d] / a.df) * lq_half;
              else
                lqs += -0.5 * e[d] * e[d] - 0.5 * kLog2Pi;
            }
          }
          if (need_lq && pre_lq) lqs = tl;
          row_of(e, lqs);
        }
      }
    } else if constexpr (HOST) {
      for (int n = tid; n < N; n += RT) {
        const long long rix = ((long long)prob * a.n_steps + s) * N + n;
        const double* row = a.noise + rix * D;
        double e[DMAX];
        double lqs = 0.0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          // the index is clamped so that no load (the compiler may issue it
          // unconditionally for the select) reads past the sample's D values,
          // i.e. past the end of the noise array for the last sample
          const double t = row[d < D ? d : D - 1];
          e[d] = d < D ? t : 0.0;
          if (need_lq && !pre_lq && d < D) {
            if constexpr (TFAM)
              lqs += a.t_const - log1p(e[d] * e[d] / a.df) * lq_half;
            else
              lqs += -0.5 * e[d] * e[d] - 0.5 * kLog2Pi;
          }
        }
        if (need_lq && pre_lq) lqs = a.noise_lq[rix];
        row_of(e, lqs);
      }
    } else {
      auto consume = [&](const double* buf, int nbase, int nc) {
        for (int n = tid; n < nc; n += RT) {
          const double* rec = buf + n * R;
          double e[DMAX];
          // unconditional loads + selects (see the step prologue); rec + d stays
          // inside s_e (DMAX doubles of slack after the record area)
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            const double t = rec[d];
            e[d] = d < D ? t : 0.0;
          }
          double lqs = 0.0;
          if (need_lq)
            for (int j = 0; j < NP; ++j) lqs += rec[2 * NP + j];
          row_of(e, lqs);
        }
        (void)nbase;
      };
      if (L.pipe) {
        double* cur = s_e + (s & 1) * (kBlockDrawLds / 2);
        double* nxt = s_e + ((s + 1) & 1) * (kBlockDrawLds / 2);
        if (rows)
          consume(cur, 0, N);
        else if (s + 1 < a.n_steps)
          draw_item(tid - RT, NT - RT, cut_a, 0, ri + 1, nxt);
        VB_PH(2);
      } else {
        const int CH = kBlockDrawLds / R;  // samples per draw chunk
        for (int c0n = 0; c0n < N; c0n += CH) {
          const int nc = min(CH, N - c0n);
          draw_item(tid, NT, nc * NP, c0n, ri, s_e);
          VB_PH(1);
          __syncthreads();
          if (rows) consume(s_e, c0n, nc);
          VB_PH(2);
          if (c0n + CH < N) __syncthreads();  // s_e is refilled by the next chunk
        }
      }
    }

    VB_BT(0);
    double M = 0.0;
    if (k_chivi) {
      if (rows) {
        const double wm = wave_max_dpp(mloc);
        if (lane == 0) s_max[wid] = wm;
      }
      __syncthreads();
      {
        double mq[kBlockMaxRowWaves];
#pragma unroll
        for (int q = 0; q < kBlockMaxRowWaves; ++q) mq[q] = s_max[q];
        M = mq[0];
#pragma unroll
        for (int q = 1; q < kBlockMaxRowWaves; ++q) M = q < RW ? fmax_raw(M, mq[q]) : M;
      }
      if (rows) {
        const double f = (mloc == -INFINITY) ? 0.0 : exp_fast(a.alpha * (mloc - M));
        if constexpr (SPLIT) {
#pragma unroll
          for (int k = 0; k < KH; ++k) acch[k] *= f;
        } else {
#pragma unroll
          for (int k = 0; k <= 2 * DMAX; ++k) acc[k] *= f;
        }
      }
    }
    VB_PH(3);
    VB_BT(1);
    if constexpr (SPLIT) {
      if (rows) wave_reduce_scatter_pair<KH, DH, DMAX>(acch, s_red[wid]);
    } else {
      if (rows) wave_reduce_scatter<K>(acc, s_red[wid]);
    }
    VB_BT(2);
    __syncthreads();
    VB_BT(3);
    // block total of column k: the row waves' rows summed in order by each reader
    // (the update threads and the value thread read their own columns, so no
    // separate column pass and barrier)
    // (every row's value is read at once, then summed in row order: a loop over
    // RW issued one dependent LDS read per row, ~0.25 us of the update's chain at
    // RW = 4)
    auto colsum = [&](int k) {
      double t[kBlockMaxRowWaves];
#pragma unroll
      for (int q = 0; q < kBlockMaxRowWaves; ++q) t[q] = s_red[q][k];
      // (the absent waves' rows hold zeros, set before the step loop: u + 0 = u)
      double u = t[0];
#pragma unroll
      for (int q = 1; q < kBlockMaxRowWaves; ++q) u = u + t[q];
      return u;
    };
    VB_PH(4);

    // gradient + update: thread p owns parameter p (wave 0, a row wave)
    if (RO != 2 && tid < P) {
      const int p = tid;
      // one column read and one division for both parameter kinds (the two
      // sides of a select, not of a branch: wave 0 holds both kinds)
      const bool mean = p < D;
      const int kc = mean ? p : DMAX + (p - D);
      const double sgp = s_sg[mean ? 0 : p - D];
      double gp;
      if (!k_chivi) {
        const double cd = colsum(kc) * inv_dN;
        gp = mean ? -cd : -(1.0 + sgp * cd);
      } else {
        // both columns' reads in flight together (the empty asm holds them until all
        // eight are loaded): the compiler had moved the weight sum's reads into a branch
        // of the log-sigma lanes after the first column's adds, then into the same
        // registers -- two LDS round trips on the update's chain instead of one
        double tc[kBlockMaxRowWaves], ts[kBlockMaxRowWaves];
#pragma unroll
        for (int q = 0; q < kBlockMaxRowWaves; ++q) {
          tc[q] = s_red[q][kc];
          ts[q] = s_red[q][2 * DMAX];
        }
        static_assert(kBlockMaxRowWaves == 4, "the asm operand list below");
        asm volatile("" : "+v"(tc[0]), "+v"(tc[1]), "+v"(tc[2]), "+v"(tc[3]), "+v"(ts[0]),
                          "+v"(ts[1]), "+v"(ts[2]), "+v"(ts[3]));
        double c = tc[0], Ssum = ts[0];
#pragma unroll
        for (int q = 1; q < kBlockMaxRowWaves; ++q) {
          c = c + tc[q];
          Ssum = Ssum + ts[q];
        }
        gp = (mean ? a.alpha * c : a.alpha * (sgp * c + Ssum)) * inv_dN;
      }
      if (k_emit) {
        a.grad[(long long)prob * P + p] = gp;
      } else {
        double nl;
        if (k_opt != 0) {
          // RMSProp-IA (vb.py:436-453) / Adam-IA (vb.py:606-617): state in
          // s_ring[0..P) (second moment) and s_ring[P..2P) (first moment); the
          // history keeps the PRE-update parameters of the last n_hist iterations.
          const double old = s_lam[p];
          if (i >= a.hist_start) a.hist[((long long)prob * a.n_hist + (i - a.hist_start)) * P + p] = old;
          const double g2 = __dmul_rn(gp, gp);
          if (k_opt == 1) {
            const double sgs = i == 0 ? g2 : __dadd_rn(__dmul_rn(s_ring[p], 0.9), __dmul_rn(1.0 - 0.9, g2));
            s_ring[p] = sgs;
            nl = __dsub_rn(old, __dmul_rn(a.lr.at(i), gp) / sqrt(__dadd_rn(a.eps, sgs)));
          } else {
            const double v = i == 0 ? __dmul_rn(0.9, g2)
                                    : __dadd_rn(__dmul_rn(s_ring[p], 0.999), __dmul_rn(1.0 - 0.999, g2));
            const double m = i == 0 ? __dmul_rn(0.9, gp)
                                    : __dadd_rn(__dmul_rn(s_ring[P + p], 0.9), __dmul_rn(1.0 - 0.9, gp));
            s_ring[p] = v;
            s_ring[P + p] = m;
            const double mh = m / (1.0 - pow(0.9, (double)(i + 2)));
            const double vh = v / (1.0 - pow(0.999, (double)(i + 2)));
            nl = __dsub_rn(old, __dmul_rn(a.lr.at(i), mh) / sqrt(__dadd_rn(a.eps, vh)));
          }
        } else {
          s_ring[slot * P + p] = gp;
          double q = 0.0;
          if (qpre) {
            if (qnext && s > 0)
              q = __dadd_rn(__dadd_rn(k_chivi ? qo_pre : s_qpre[s & 1][p], __dmul_rn(gprev, gprev)),
                            __dmul_rn(gp, gp));
            else
              q = __dadd_rn(s_qold[p], __dmul_rn(gp, gp));
            gprev = gp;
          } else {
            const int cnt = (i + 1 < W) ? (int)(i + 1) : W;
            const int oldest = (cnt < W || slot + 1 == W) ? 0 : slot + 1;  // (i + 1) % W
            for (int k = 0; k < cnt; ++k) {
              int Lk = oldest + k;
              if (Lk >= W) Lk -= W;
              const double t = s_ring[Lk * P + p];
              q = __dadd_rn(q, __dmul_rn(t, t));
            }
          }
          // lam - lr g / sqrt(eps + q) with the refined rsqrt of the column-pair
          // kernel's update (~1 ulp) instead of an IEEE sqrt and division: ~30
          // instructions off the step's serial update chain
          const double lr_u = k_chivi ? lr_i : a.lr.at(i);
          nl = __dsub_rn(s_lam[p], __dmul_rn(lr_u, gp) * rsqrt_pos(__dadd_rn(a.eps, q)));
          if (i >= a.hist_start) a.hist[((long long)prob * a.n_hist + (i - a.hist_start)) * P + p] = nl;
        }
        s_lam[p] = nl;  // only thread p reads/writes s_lam[p] / s_sg[p - D] until the barrier
        if (p >= D) s_sg[p - D] = exp_fast(nl);
      }
    }
    if (RO != 1 && tid == val_tid) {
      double val;
      if constexpr (kPF) sl = s_sl;
      if (!k_chivi) {
        // entropy uses the pre-update lam: sum_d log sigma_d (the sampled log q of
        // klvi_pd lacks it: -(mean (log p - log q)) = -(st / N + sl))
        const double st = colsum(2 * DMAX);
        val = k_pd ? -(st / dN + sl) : -(c0 + sl + st / dN);
      } else {
        val = log(colsum(2 * DMAX) / dN) / a.alpha + (M + sl);
      }
      a.values[(long long)prob * a.n_iters + (k_emit ? 0 : i)] = val;
    }
    if constexpr (!HOST) {
      // the draw waves' last item round of step s + 1 runs here, beside the
      // update (one row wave's P threads), instead of lengthening the
      // consume phase they already bound
      if (L.pipe && !rows && cut_a < N * NP && s + 1 < a.n_steps)
        draw_item(cut_a + tid - RT, NT - RT, N * NP, 0, ri + 1,
                  s_e + ((s + 1) & 1) * (kBlockDrawLds / 2));
    }
    VB_PH(5);
    VB_BT(4);
    slot = slot + 1 == W ? 0 : slot + 1;
    __syncthreads();
    VB_PH(6);
    VB_BT(5);
  };
  // (the t family runs only with pre-drawn noise: one loop of row waves)
  bool split = false;
  if constexpr (!HOST && !TFAM) split = L.pipe;
  if (copy_wave) {
    // The copy wave's own loop: per step, wait for its last prefetch (step s + 1,
    // issued one step ago, so it has landed before this wave's first barrier of
    // step s), stage step s + 2 into slot (s + 2) % 3 (read in step s - 1, before
    // that step's last barrier), then join the step's barriers -- raw s_barrier:
    // __syncthreads' release fence would wait for the new prefetch (vmcnt(0))
    // and hold every wave at the step's first barrier.  The count matches the
    // row waves' step: the CHIVI max barrier, the reduction barrier and the
    // end-of-step barrier.
    // It also writes the window sums of step s (s_qold) before the step's first
    // barrier: the slots it reads were written by earlier steps' updates (before
    // their end barriers), and the update of step s reads s_qold after the
    // reduction barrier.
    const int nbar = k_chivi ? 3 : 2;
    int cslot = slot;
#ifdef VB_BLOCK_TS
    // the copy wave's own marks (lane 0 of problem 0): prefetch landed, prefetch
    // issued, window sums done, log-sigma sum + LDS drained, first barrier left
    unsigned long long ct[5] = {0, 0, 0, 0, 0}, tc = clock64();
#define VB_CT(k) do { const unsigned long long t_ = clock64(); ct[k] += t_ - tc; tc = t_; } while (0)
#else
#define VB_CT(k) do {} while (0)
#endif
    for (int s = 0; s < a.n_steps; ++s) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      VB_CT(0);
      if (s + 2 < a.n_steps) pf_issue(s + 2);
      VB_CT(1);
      // the window sums (s_qold) and sum_d log sigma_d (s_sl) of step s: both are first
      // read after the step's reduction barrier (CHIVI form, below)
      auto presums = [&]() __attribute__((always_inline)) {
        if (qpre && lane < P) {
          const long long i = a.step0 + s;
          const int cnt = (i + 1 < W) ? (int)(i + 1) : W;
          const int oldest = (cnt < W || cslot + 1 == W) ? 0 : cslot + 1;
          double q = 0.0;
          for (int k = 0; k + 1 < cnt; ++k) {
            int Lk = oldest + k;
            if (Lk >= W) Lk -= W;
            const double t = s_ring[Lk * P + lane];
            q = __dadd_rn(q, __dmul_rn(t, t));
          }
          s_qold[lane] = q;
        }
        VB_CT(2);
        cslot = cslot + 1 == W ? 0 : cslot + 1;
        if (lane == 0) {   // sum_d log sigma_d for the value (same order as the rows' loop)
          double sl = 0.0;
  #pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            const double l = s_lam[D + d];
            sl += d < D ? l : 0.0;
          }
          s_sl = sl;
        }
      };
      if (k_chivi) {
        // CHIVI: sum_d log sigma_d (and at a run's first step, or without qnext, the
        // window sums) after the block-max barrier, beside the rows' rescale and
        // reduce-scatter, instead of holding that barrier (the copy wave arrived last
        // there: profiles/r05/copy_wave_ts.log); s_lam is still the pre-update lambda
        // until the reduction barrier.  With qnext the next step's window sums run after
        // the reduction barrier, beside the update (below).  (KLVI keeps its code in a
        // separate copy: sharing one lambda changed the KLVI instances' code and cost
        // config 1 3 %.)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        VB_CT(3);
        __builtin_amdgcn_s_barrier();   // the block-max barrier
        VB_CT(4);
        if (!(qnext && s > 0)) {
          presums();
        } else {
          cslot = cslot + 1 == W ? 0 : cslot + 1;
          if (lane == 0) {   // sum_d log sigma_d for the value (same order as the rows' loop)
            double sl = 0.0;
#pragma unroll
            for (int d = 0; d < DMAX; ++d) {
              const double l = s_lam[D + d];
              sl += d < D ? l : 0.0;
            }
            s_sl = sl;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (qnext) {
          __builtin_amdgcn_s_barrier();   // the reduction barrier
          if (lane < P && s + 1 < a.n_steps) {
            // as KLVI's qnext below: step s + 1's older slots but the newest, oldest first
            const long long i1 = a.step0 + s + 1;
            const int cnt = (i1 + 1 < W) ? (int)(i1 + 1) : W;
            const int oldest = (cnt < W || cslot + 1 == W) ? 0 : cslot + 1;
            double q = 0.0;
            for (int k = 0; k + 2 < cnt; ++k) {
              int Lk = oldest + k;
              if (Lk >= W) Lk -= W;
              const double t = s_ring[Lk * P + lane];
              q = __dadd_rn(q, __dmul_rn(t, t));
            }
            s_qpre[(s + 1) & 1][lane] = q;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          __builtin_amdgcn_s_barrier();   // the end-of-step barrier
#ifdef VB_BLOCK_TS
          tc = clock64();
#endif
          continue;
        }
      } else {
        if (qpre && lane < P && !(qnext && s > 0)) {
          const long long i = a.step0 + s;
          const int cnt = (i + 1 < W) ? (int)(i + 1) : W;
          const int oldest = (cnt < W || cslot + 1 == W) ? 0 : cslot + 1;
          double q = 0.0;
          for (int k = 0; k + 1 < cnt; ++k) {
            int Lk = oldest + k;
            if (Lk >= W) Lk -= W;
            const double t = s_ring[Lk * P + lane];
            q = __dadd_rn(q, __dmul_rn(t, t));
          }
          s_qold[lane] = q;
        }
        VB_CT(2);
        cslot = cslot + 1 == W ? 0 : cslot + 1;
        if (lane == 0) {   // sum_d log sigma_d for the value (same order as the rows' loop)
          double sl = 0.0;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            const double l = s_lam[D + d];
            sl += d < D ? l : 0.0;
          }
          s_sl = sl;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        VB_CT(3);
        __builtin_amdgcn_s_barrier();   // the reduction barrier
        VB_CT(4);
        if (qnext && lane < P && s + 1 < a.n_steps) {
          // step s + 1's older window slots but the newest (step s's, written by the
          // update running now), oldest first; cslot is already step s + 1's slot.  The
          // slots read were written by step s - 1's update or earlier; step s's update
          // writes the slot of step s + 1 - W, which is not among them.
          const long long i1 = a.step0 + s + 1;
          const int cnt = (i1 + 1 < W) ? (int)(i1 + 1) : W;
          const int oldest = (cnt < W || cslot + 1 == W) ? 0 : cslot + 1;
          double q = 0.0;
          for (int k = 0; k + 2 < cnt; ++k) {
            int Lk = oldest + k;
            if (Lk >= W) Lk -= W;
            const double t = s_ring[Lk * P + lane];
            q = __dadd_rn(q, __dmul_rn(t, t));
          }
          s_qpre[(s + 1) & 1][lane] = q;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
      for (int b = 1; b < nbar; ++b) __builtin_amdgcn_s_barrier();
#ifdef VB_BLOCK_TS
      tc = clock64();   // (the step's later barriers not counted)
#endif
    }
#ifdef VB_BLOCK_TS
    if (prob == 0 && lane == 0 && a.n_steps > 0)
      printf("COPYTS hw_id=0x%x steps=%d | vmcnt wait %.0f issue %.0f window sums %.0f log-sigma sum + drain %.0f first barrier wait %.0f\n",
             (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)), a.n_steps, (double)ct[0] / a.n_steps, (double)ct[1] / a.n_steps, (double)ct[2] / a.n_steps,
             (double)ct[3] / a.n_steps, (double)ct[4] / a.n_steps);
#endif
#undef VB_CT
  } else if (split) {
    if constexpr (!HOST && !TFAM) {
      if (row_wave) {
        for (int s = 0; s < a.n_steps; ++s) step(s, std::integral_constant<int, 1>{});
      } else {
        for (int s = 0; s < a.n_steps; ++s) step(s, std::integral_constant<int, 2>{});
      }
    }
  } else {
    for (int s = 0; s < a.n_steps; ++s) step(s, std::integral_constant<int, 0>{});
  }
#ifdef VB_BLOCK_PROF
  if (prob == 0 && (tid == 0 || tid == RT)) {  // a row wave and the first draw wave
    const unsigned long long tw = wall_clock64() - tw0, tc = clock64() - tc0;
    printf("BLOCKPROF tid=%d D=%d N=%d NT=%d RW=%d pipe=%d steps=%d wall_ticks=%llu cycles=%llu | exp %llu draw %llu row %llu chivi %llu bsum %llu upd %llu bar %llu\n",
           tid, D, N, NT, RW, L.pipe, a.n_steps, tw, tc, ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], ph[6]);
  }
#endif
#undef VB_PH
#ifdef VB_BLOCK_TS
  if (prob == 0 && lane == 0 && row_wave && a.n_steps > 0)
    printf("BLOCKTS wave=%d hw_id=0x%x D=%d N=%d NT=%d RW=%d chivi=%d steps=%d cyc/step=%.0f | rows %.0f max+bar %.0f rs %.0f bar %.0f upd %.0f bar %.0f\n",
           wid, (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11)), D, N, NT, RW, k_chivi ? 1 : 0, a.n_steps, (double)(clock64() - tb0) / a.n_steps,
           (double)bt[0] / a.n_steps, (double)bt[1] / a.n_steps, (double)bt[2] / a.n_steps,
           (double)bt[3] / a.n_steps, (double)bt[4] / a.n_steps, (double)bt[5] / a.n_steps);
#endif
#undef VB_BT

  if (!k_emit) {
    for (int p = tid; p < P; p += NT) lam_g[p] = s_lam[p];
    for (int q = tid; q < W * P; q += NT) ring_g[q] = s_ring[q];
  }
}

// Latency floor of the block kernel's step (measurement only, vb_block_floor):
// the same block shape, barriers, reductions and adagrad update as block_kernel,
// with no draws and no target -- every row thread's accumulators are a cheap
// function of the current parameters (so each step still depends on the last
// update).  Its time per step bounds what any block_kernel step can reach.
template <int DMAX>
__global__ __launch_bounds__(kBlockMaxThreads) void block_floor_kernel(int D, int N, int NT_rows,
                                                                     int chivi, int n_steps,
                                                                     int W, double* out, int n_act,
                                                                     int has_copy) {
  constexpr int K = 2 * DMAX + 2;
  __shared__ double s_lam[2 * DMAX];
  __shared__ double s_sg[DMAX];
  __shared__ double s_ring[64 * 2 * DMAX];
  __shared__ double s_red[kBlockMaxRowWaves][K];
  __shared__ double s_max[kBlockMaxRowWaves];
  // window pre-sums, parity-indexed as block_kernel's s_qpre: KLVI's copy wave
  // writes step s + 1's while the update threads read step s's
  __shared__ double s_qpre[2][2 * DMAX];
  __shared__ double s_sl;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int NT = blockDim.x, P = 2 * D, RW = NT_rows / 64;
  const bool row_wave = wid < RW;
  // the copy-wave layout: that wave pre-sums the window and sum_d log sigma_d, as
  // block_kernel's copy wave does
  const bool copy = has_copy && wid == RW, qpre = has_copy && W <= kBlockQpreMaxW;
  const double dN = (double)N;
  for (int p = tid; p < P; p += NT) s_lam[p] = 0.01 * p;
  for (int q = tid; q < W * P; q += NT) s_ring[q] = 0.0;
  for (int d = tid; d < D; d += NT) s_sg[d] = 1.0;
  for (int p = tid; p < 2 * 2 * DMAX; p += NT) (&s_qpre[0][0])[p] = 0.0;
  for (int q = RW * K + tid; q < kBlockMaxRowWaves * K; q += NT) (&s_red[0][0])[q] = 0.0;
  __syncthreads();
  int slot = 0;
  double val = 0.0, gprev = 0.0;
  const double inv_dN = 1.0 / dN;
  // ring slots of steps [first, first + n), oldest first, squared and summed into
  // buf (the copy wave, lanes < P)
  auto window_sum = [&](int first, int n, double* buf) {
    if (qpre && lane < P) {
      double q = 0.0;
      int L = first % W;
      for (int k = 0; k < n; ++k) {
        const double v = s_ring[L * P + lane];
        q = __dadd_rn(q, __dmul_rn(v, v));
        L = L + 1 == W ? 0 : L + 1;
      }
      buf[lane] = q;
    }
  };
  for (int s = 0; s < n_steps; ++s) {
    // (as block_kernel: CHIVI reads the window pre-sum at the step's start, KLVI after
    // the reduction barrier)
    const double qo_pre = (chivi && qpre && tid < P) ? s_qpre[s & 1][tid] : 0.0;
    double sl = 0.0;
    if (!has_copy || copy) {
#pragma unroll
      for (int d = 0; d < DMAX; ++d) sl += d < D ? s_lam[D + d] : 0.0;
    }
    // (block_kernel's copy wave: sum_d log sigma_d before the reduction barrier, the
    // NEXT step's window but its two newest slots after the reduction barrier, beside
    // the update -- qnext, KLVI and CHIVI)
    if (copy && lane == 0) s_sl = sl;
    // accumulators: a cheap function of the last update (one LDS read and K adds; a
    // per-k read of s_lam[k % P] spent an integer division per accumulator and made
    // the floor grow with K by ~0.06 us per accumulator)
    double acc[K];
    const double t = (double)(tid + 1) * 1e-3 * s_lam[0];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = (tid < n_act) ? t + (double)k : 0.0;
    double M = 0.0;
    if (chivi) {
      if (row_wave) {
        const double wm = wave_max_dpp(tid < n_act ? t : -INFINITY);
        if (lane == 0) s_max[wid] = wm;
      }
      __syncthreads();
      double mq[kBlockMaxRowWaves];
#pragma unroll
      for (int q = 0; q < kBlockMaxRowWaves; ++q) mq[q] = s_max[q];
      M = mq[0];
#pragma unroll
      for (int q = 1; q < kBlockMaxRowWaves; ++q) M = q < RW ? fmax(M, mq[q]) : M;
    }
    if (row_wave) wave_reduce_scatter<K>(acc, s_red[wid]);
    __syncthreads();
    if (copy) {
      // step s + 1's window (min(s + 2, W) slots) without steps s and s + 1
      const int cnt1 = s + 2 < W ? s + 2 : W;
      window_sum(s + 2 - cnt1, cnt1 - 2, s_qpre[(s + 1) & 1]);
    }
    auto colsum = [&](int k) {   // as block_kernel: each reader sums its column
      double tq[kBlockMaxRowWaves];
#pragma unroll
      for (int q = 0; q < kBlockMaxRowWaves; ++q) tq[q] = s_red[q][k];
      double u = tq[0];
#pragma unroll
      for (int q = 1; q < kBlockMaxRowWaves; ++q) u = u + tq[q];   // (absent rows: zeros)
      return u;
    };
    if (tid < P) {
      const int p = tid;
      const bool mean = p < D;
      const double cd = colsum(mean ? p : DMAX + (p - D)) * inv_dN;
      const double gp = mean ? -cd : -(1.0 + s_sg[mean ? 0 : p - D] * cd);
      s_ring[slot * P + p] = gp;
      double q = 0.0;
      if (qpre) {
        const double qo = chivi ? qo_pre : s_qpre[s & 1][p];
        q = s > 0 ? __dadd_rn(__dadd_rn(qo, __dmul_rn(gprev, gprev)), __dmul_rn(gp, gp))
                  : __dadd_rn(qo, __dmul_rn(gp, gp));
        gprev = gp;
      } else {
        const int cnt = (s + 1 < W) ? s + 1 : W;
        const int oldest = (cnt < W || slot + 1 == W) ? 0 : slot + 1;
        for (int k = 0; k < cnt; ++k) {
          int Lk = oldest + k;
          if (Lk >= W) Lk -= W;
          const double v = s_ring[Lk * P + p];
          q = __dadd_rn(q, __dmul_rn(v, v));
        }
      }
      const double nl = __dsub_rn(s_lam[p], __dmul_rn(1e-6, gp) * rsqrt_pos(__dadd_rn(0.1, q)));
      s_lam[p] = nl;
      if (p >= D) s_sg[p - D] = exp_fast(nl);
    }
    if (tid == (NT > 64 ? NT - 64 : 0)) {
      if (has_copy) sl = s_sl;
      val += chivi ? log(colsum(2 * DMAX) / dN) + M + sl : colsum(2 * DMAX) + sl;
    }
    slot = slot + 1 == W ? 0 : slot + 1;
    __syncthreads();
  }
  if (tid == (NT > 64 ? NT - 64 : 0)) out[blockIdx.x] = val;
}

hipError_t launch_block_floor(int D, int N, bool host_layout, bool chivi, int n_steps, int nprob,
                              double* out, hipStream_t s, int pf) {
  if (D < 1 || D > kBlockDMax || N < 1 || n_steps < 0 || nprob < 1) return hipErrorInvalidValue;
  // the same block shape as block_kernel's (with the device-noise copy wave, which
  // only joins the barriers here)
  const BlockLayout L = block_layout(N, D, host_layout, chivi, pf);
  const dim3 grid(nprob), block(L.nt);
  // (split rows: 2N active row lanes, each reducing the full K accumulators -- an
  // upper bound on the split kernel's KH-wide pair reduction)
  const int rows = 64 * L.rw, W = 10, n_act = L.split ? 2 * N : N;
  if (D <= 2)
    hipLaunchKernelGGL((block_floor_kernel<2>), grid, block, 0, s, D, N, rows, chivi ? 1 : 0, n_steps, W, out, n_act, L.pf);
  else if (D <= 4)
    hipLaunchKernelGGL((block_floor_kernel<4>), grid, block, 0, s, D, N, rows, chivi ? 1 : 0, n_steps, W, out, n_act, L.pf);
  else if (D <= 10)
    hipLaunchKernelGGL((block_floor_kernel<10>), grid, block, 0, s, D, N, rows, chivi ? 1 : 0, n_steps, W, out, n_act, L.pf);
  else
    hipLaunchKernelGGL((block_floor_kernel<kBlockDMax>), grid, block, 0, s, D, N, rows, chivi ? 1 : 0, n_steps, W, out, n_act, L.pf);
  return hipGetLastError();
}

// Pre-drawn noise for the block kernel's device-noise path (launch_block_predraw):
// one thread per (problem, step, sample) walks the sample's column pairs with the
// draw items' counters, transforms and log q partials (block_kernel's draw_item),
// so the block kernel consuming it computes bit-identical results to drawing in
// kernel -- while the draws, which never depend on lambda, run as a throughput
// kernel over the whole chip instead of on the serial step chain of one
// workgroup per problem.
template <bool TFAM>
__global__ __launch_bounds__(256) void block_predraw_kernel(int D, int N, int n_steps, long long total,
                                                            uint32_t k0, uint32_t k1, uint32_t stream,
                                                            uint32_t stride, long long rng_step0,
                                                            double t_scale, double shape, double df,
                                                            double t_const, double* noise,
                                                            double* lq) {
  __shared__ double2 s_sct[kSinCosN];
  __shared__ double2 s_lt[kLogN + kLogU01N];
  load_bm_tables(s_sct, s_lt);
  __syncthreads();
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;  // (q * n_steps + s) * N + n
  if (idx >= total) return;
  const int n = (int)(idx % N);
  const long long qs = idx / N;
  const int s = (int)(qs % n_steps);
  const uint32_t q = (uint32_t)(qs / n_steps);
  const Rng rng{k0, k1, stream + q * stride};
  const uint32_t ri = (uint32_t)(rng_step0 + s);
  const int NP = (D + 1) / 2;
  const double lq_half = 0.5 * (df + 1.0);
  const double inv_df = 1.0 / df;
  double* row = noise + idx * D;
  double lqs = 0.0;
  for (int j = 0; j < NP; ++j) {
    double ea, eb;
    normal_pair_tab(rng.draw((uint32_t)j, (uint32_t)n, ri, 0u), ea, eb, s_sct, s_lt);
    if constexpr (TFAM) {
      double ga, gb;
      gamma_pair<true>(rng, (uint32_t)j, (uint32_t)n, ri, shape, ga, gb, s_sct, s_lt);
      ea = t_scale * ea * rsqrt_pos(ga);
      eb = t_scale * eb * rsqrt_pos(gb);
    }
    const bool hasb = 2 * j + 1 < D;
    row[2 * j] = ea;
    if (hasb) row[2 * j + 1] = eb;
    if (lq) {
      double lqp;
      if constexpr (TFAM) {
        lqp = t_const - log1p_pos_tab(ea * ea * inv_df, s_lt) * lq_half;
        if (hasb) lqp += t_const - log1p_pos_tab(eb * eb * inv_df, s_lt) * lq_half;
      } else {
        lqp = -0.5 * ea * ea - 0.5 * kLog2Pi;
        if (hasb) lqp += -0.5 * eb * eb - 0.5 * kLog2Pi;
      }
      lqs += lqp;
    }
  }
  if (lq) lq[idx] = lqs;
}

hipError_t launch_block_predraw(int fam, int D, int N, int n_steps, int nprob, uint32_t k0,
                                uint32_t k1, uint32_t stream, uint32_t stride, long long rng_step0,
                                double t_scale, double shape, double df, double t_const,
                                double* noise, double* lq, hipStream_t s) {
  const long long total = (long long)nprob * n_steps * N;
  if (total <= 0) return hipSuccess;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (fam == 1)
    hipLaunchKernelGGL(block_predraw_kernel<true>, grid, dim3(256), 0, s, D, N, n_steps, total, k0,
                       k1, stream, stride, rng_step0, t_scale, shape, df, t_const, noise, lq);
  else
    hipLaunchKernelGGL(block_predraw_kernel<false>, grid, dim3(256), 0, s, D, N, n_steps, total, k0,
                       k1, stream, stride, rng_step0, t_scale, shape, df, t_const, noise, lq);
  return hipGetLastError();
}

// -------------------------------------------------------------------------
// elementwise helpers
// -------------------------------------------------------------------------
template <bool TFAM, bool HOST>
__global__ __launch_bounds__(256) void sample_kernel(int D, long long n, const double* lam,
                                                     double t_scale, double shape,
                                                     const double* noise, Rng rng,
                                                     uint32_t step, double* x) {
  const int npairs = (D + 1) / 2;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * npairs) return;
  const long long r = idx / npairs;
  const int j = (int)(idx % npairs);
  const int dA = 2 * j, dB = 2 * j + 1;
  double eA, eB;
  if constexpr (HOST) {
    eA = noise[r * D + dA];
    eB = dB < D ? noise[r * D + dB] : 0.0;
  } else {
    normal_pair(rng.draw((uint32_t)j, (uint32_t)r, step, 0u), eA, eB);
    if constexpr (TFAM) {
      double ga, gb;
      gamma_pair(rng, (uint32_t)j, (uint32_t)r, step, shape, ga, gb);
      eA = t_scale * eA / sqrt(ga);
      eB = t_scale * eB / sqrt(gb);
    }
  }
  x[r * D + dA] = eA * exp(lam[D + dA]) + lam[dA];
  if (dB < D) x[r * D + dB] = eB * exp(lam[D + dB]) + lam[dB];
}

// one wavefront per row: out[r] = sum_d log q_d(x[r, d])
template <bool TFAM>
__global__ __launch_bounds__(256) void family_logdensity_kernel(int D, long long n,
                                                                const double* lam, double df,
                                                                double t_const, const double* x,
                                                                double* out) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int d = lane; d < D; d += 64) {
    const double ls = lam[D + d];
    const double z = (x[r * D + d] - lam[d]) / exp(ls);
    if constexpr (TFAM)
      acc += t_const - log1p(z * z / df) * (0.5 * (df + 1.0)) - ls;
    else
      acc += -0.5 * z * z - ls - 0.5 * kLog2Pi;
  }
  acc = wave_sum(acc);
  if (lane == 0) out[r] = acc;
}

template <class TGT>
__global__ __launch_bounds__(256) void target_sep_kernel(int D, long long n, const double* x,
                                                         double* out, double* grad) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
  for (int d = lane; d < D; d += 64) {
    double g;
    acc += TGT::lp1(x[r * D + d], g);
    if (grad) grad[r * D + d] = g;
  }
  acc = wave_sum(acc);
  if (lane == 0) out[r] = acc;
}

// Funnel at any D: one wavefront per row (x[1] = log sigma broadcast to the row).
__global__ __launch_bounds__(256) void funnel_wide_kernel(int D, long long n, const double* x,
                                                          double* out, double* grad) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  constexpr double s0 = 1.35;
  const double v = x[r * D + 1];
  const double scale = exp(v), inv_s2 = exp(-2.0 * v);
  double lp = 0.0, gv = 0.0;
  for (int d = lane; d < D; d += 64) {
    if (d == 1) continue;
    const double xd = x[r * D + d];
    const double z = xd / scale;
    lp += -0.5 * z * z - v - 0.5 * kLog2Pi;
    if (grad) grad[r * D + d] = -xd * inv_s2;
    gv += z * z - 1.0;
  }
  lp = wave_sum(lp);
  gv = wave_sum(gv);
  if (lane == 0) {
    const double zv = v / s0;
    out[r] = (-0.5 * zv * zv - log(s0) - 0.5 * kLog2Pi) + lp;
    if (grad) grad[r * D + 1] = -zv / s0 + gv;
  }
}

// ---- wide rows (D >= kWideRowD, few rows): one 1024-thread block per row --------
// The one-wavefront-per-row kernels above suit many short rows (log weights: m
// rows of D <= 16 or so); a step of the materialised mean-field path has N ~ 100
// rows of D ~ 1e4, where one wave per row leaves the chip ~90 % idle.  Fixed-order
// block reductions keep the sums deterministic.
constexpr int kWideRowD = 512;

__device__ __forceinline__ double block_sum_1024(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) t += red[q];
  __syncthreads();
  return t;
}

template <bool TFAM>
__global__ __launch_bounds__(1024) void family_logdensity_rowblock_kernel(int D, const double* lam,
                                                                         double df, double t_const,
                                                                         const double* x,
                                                                         double* out) {
  __shared__ double red[16];
  const long long r = blockIdx.x;
  double acc = 0.0;
  for (int d = threadIdx.x; d < D; d += 1024) {
    const double ls = lam[D + d];
    const double z = (x[r * D + d] - lam[d]) / exp(ls);
    if constexpr (TFAM)
      acc += t_const - log1p(z * z / df) * (0.5 * (df + 1.0)) - ls;
    else
      acc += -0.5 * z * z - ls - 0.5 * kLog2Pi;
  }
  acc = block_sum_1024(acc, red);
  if (threadIdx.x == 0) out[r] = acc;
}

template <class TGT>
__global__ __launch_bounds__(1024) void target_sep_rowblock_kernel(int D, const double* x,
                                                                  double* out, double* grad) {
  __shared__ double red[16];
  const long long r = blockIdx.x;
  double acc = 0.0;
  for (int d = threadIdx.x; d < D; d += 1024) {
    double g;
    acc += TGT::lp1(x[r * D + d], g);
    if (grad) grad[r * D + d] = g;
  }
  acc = block_sum_1024(acc, red);
  if (threadIdx.x == 0) out[r] = acc;
}

__global__ __launch_bounds__(1024) void funnel_rowblock_kernel(int D, const double* x, double* out,
                                                               double* grad) {
  __shared__ double red[16];
  const long long r = blockIdx.x;
  constexpr double s0 = 1.35;
  const double v = x[r * D + 1];
  const double scale = exp(v), inv_s2 = exp(-2.0 * v);
  double lp = 0.0, gv = 0.0;
  for (int d = threadIdx.x; d < D; d += 1024) {
    if (d == 1) continue;
    const double xd = x[r * D + d];
    const double z = xd / scale;
    lp += -0.5 * z * z - v - 0.5 * kLog2Pi;
    if (grad) grad[r * D + d] = -xd * inv_s2;
    gv += z * z - 1.0;
  }
  lp = block_sum_1024(lp, red);
  gv = block_sum_1024(gv, red);
  if (threadIdx.x == 0) {
    const double zv = v / s0;
    out[r] = (-0.5 * zv * zv - log(s0) - 0.5 * kLog2Pi) + lp;
    if (grad) grad[r * D + 1] = -zv / s0 + gv;
  }
}

template <class TGT, int DMAX>
__global__ __launch_bounds__(256) void target_row_kernel(int D, long long n, const double* x,
                                                         double* out, double* grad) {
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  double xv[DMAX], g[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    xv[d] = d < D ? x[r * D + d] : 0.0;
    g[d] = 0.0;
  }
  out[r] = TGT::template row<DMAX>(xv, g, D);
  if (grad)
    for (int d = 0; d < D; ++d) grad[r * D + d] = g[d];
}

// scale (nullable): per window position, oldest first, the reference's
// grad_scale = exp(min(log_norms) - log_norm_j) of has_log_norm objectives
// (vb.py:371-373): accum = sum_j (scale_j g_j)^2.
__global__ __launch_bounds__(256) void adagrad_update_kernel(long long P, double* lam,
                                                             const double* g, double* ring,
                                                             int W, long long step, double lr,
                                                             double eps, const double* scale,
                                                             double* hrow) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const double v = adagrad_step(p, P, lam[p], g[p], ring, W, step, lr, eps, scale);
  lam[p] = v;
  if (hrow) hrow[p] = v;   // history row (vb.py:375-376) without a separate copy
}

__global__ __launch_bounds__(256) void ia_update_kernel(int opt, long long P, double* lam,
                                                       const double* g, double* state,
                                                       long long i, double lr, double eps,
                                                       double norm2, double* old_out) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const double old = lam[p], gp = g[p], g2 = __dmul_rn(gp, gp);
  if (old_out) old_out[p] = old;
  double nl;
  if (opt == 3) {
    // RMSProp-IA with avg_grad_norm (vb.py:443-451): one host-computed scalar
    // normaliser for every coordinate
    nl = __dsub_rn(old, __dmul_rn(lr, gp) / sqrt(__dadd_rn(eps, norm2)));
  } else if (opt == 1) {
    const double sgs = i == 0 ? g2 : __dadd_rn(__dmul_rn(state[p], 0.9), __dmul_rn(1.0 - 0.9, g2));
    state[p] = sgs;
    nl = __dsub_rn(old, __dmul_rn(lr, gp) / sqrt(__dadd_rn(eps, sgs)));
  } else {
    const double v = i == 0 ? __dmul_rn(0.9, g2)
                            : __dadd_rn(__dmul_rn(state[p], 0.999), __dmul_rn(1.0 - 0.999, g2));
    const double m = i == 0 ? __dmul_rn(0.9, gp)
                            : __dadd_rn(__dmul_rn(state[P + p], 0.9), __dmul_rn(1.0 - 0.9, gp));
    state[p] = v;
    state[P + p] = m;
    const double mh = m / (1.0 - pow(0.9, (double)(i + 2)));
    const double vh = v / (1.0 - pow(0.999, (double)(i + 2)));
    nl = __dsub_rn(old, __dmul_rn(lr, mh) / sqrt(__dadd_rn(eps, vh)));
  }
  lam[p] = nl;
}

// log weights lw[r] = log p(x_r) - log q(x_r; lam) for x_r ~ q   (experiments.py:60-63)
// Philox draws use the LDS Box-Muller tables (sct, lt; loaded by the caller's
// block) like the fused kernels.
template <bool TFAM, bool HOST>
__device__ __forceinline__ void draw_pair(const Rng& rng, const double* noise, int D, long long r,
                                          int j, uint32_t step, double t_scale, double shape,
                                          double& eA, double& eB, const double2* sct,
                                          const double2* lt) {
  const int dA = 2 * j, dB = 2 * j + 1;
  if constexpr (HOST) {
    eA = noise[r * D + dA];
    eB = dB < D ? noise[r * D + dB] : 0.0;
  } else if constexpr (TFAM) {
    // the log-weight draws of the t family: Bailey pairs (bailey_t); shape and
    // t_scale belong to the estimators' normal / gamma draws
    (void)t_scale;
    (void)shape;
    const u4 w = rng.draw((uint32_t)j, (uint32_t)r, step, kBaileyPurpose);
    const double df = 2.0 * shape, c2 = -2.0 / df;
    double l1;
    eA = bailey_t(w.x, w.z, df, c2, sct, lt, l1);
    eB = bailey_t(w.y, w.w, df, c2, sct, lt, l1);
  } else {
    normal_pair_tab(rng.draw((uint32_t)j, (uint32_t)r, step, 0u), eA, eB, sct, lt);
  }
}

// logq1 with sigma = exp(ls) given (the same bits)
template <bool TFAM, bool HOST>
__device__ __forceinline__ double logq1s(double x, double mu, double ls, double sg, double df,
                                         double t_const, const double2* lt) {
  const double z = (x - mu) / sg;
  if constexpr (TFAM) {
    const double y = z * z / df;
    double l1;
    if constexpr (HOST) l1 = log1p(y);
    else l1 = log1p_pos_tab(y, lt);
    return t_const - l1 * (0.5 * (df + 1.0)) - ls;
  }
  return -0.5 * z * z - ls - 0.5 * kLog2Pi;
}

template <bool TFAM, bool HOST>
__device__ __forceinline__ double logq1(double x, double mu, double ls, double df,
                                        double t_const, const double2* lt) {
  const double z = (x - mu) / exp(ls);
  if constexpr (TFAM) {
    const double y = z * z / df;
    double l1;
    if constexpr (HOST) l1 = log1p(y);
    else l1 = log1p_pos_tab(y, lt);
    return t_const - l1 * (0.5 * (df + 1.0)) - ls;
  }
  return -0.5 * z * z - ls - 0.5 * kLog2Pi;
}

// separable targets: one wavefront per draw, lanes over column pairs
template <class TGT, bool TFAM, bool HOST>
__global__ __launch_bounds__(256) void logw_sep_kernel(int D, long long m, const double* lam,
                                                       double t_scale, double shape, double df,
                                                       double t_const, const double* noise,
                                                       Rng rng, uint32_t step, uint32_t stride, double* lw,
                                                       double* xs) {
  __shared__ double2 s_sct[HOST ? 1 : kSinCosN];
  __shared__ double2 s_lt[HOST ? 1 : kLogN + kLogU01N];
  if constexpr (!HOST) {
    load_bm_tables(s_sct, s_lt);
    __syncthreads();
  }
  // row q of a batched launch (vb_log_weights_rows): its own lambda, output
  // row, noise rows and Philox stream (stream + q * stride)
  const int q = blockIdx.y;
  lam += (long long)q * 2 * D;
  lw += (long long)q * m;
  if (xs) xs += (long long)q * m * D;
  if (noise) noise += (long long)q * m * D;
  rng.stream += (uint32_t)q * stride;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= m) return;
  const int lane = threadIdx.x & 63, npairs = (D + 1) / 2;
  double lp = 0.0, lq = 0.0;
  for (int j = lane; j < npairs; j += 64) {
    double e[2];
    draw_pair<TFAM, HOST>(rng, noise, D, r, j, step, t_scale, shape, e[0], e[1], s_sct, s_lt);
    for (int c = 0; c < 2; ++c) {
      const int d = 2 * j + c;
      if (d < D) {
        const double mu = lam[d], ls = lam[D + d];
        const double x = e[c] * exp(ls) + mu;
        double g;
        lp += TGT::lp1(x, g);
        lq += logq1<TFAM, HOST>(x, mu, ls, df, t_const, s_lt);
        if (xs) xs[r * D + d] = x;
      }
    }
  }
  lp = wave_sum(lp);
  lq = wave_sum(lq);
  if (lane == 0) lw[r] = lp - lq;
}

// any target with D <= DMAX: one thread per draw
template <class TGT, bool TFAM, bool HOST, int DMAX>
__global__ __launch_bounds__(256) void logw_row_kernel(int D, long long m, const double* lam,
                                                       double t_scale, double shape, double df,
                                                       double t_const, const double* noise,
                                                       Rng rng, uint32_t step, uint32_t stride, double* lw,
                                                       double* xs) {
  __shared__ double2 s_sct[HOST ? 1 : kSinCosN];
  __shared__ double2 s_lt[HOST ? 1 : kLogN + kLogU01N];
  __shared__ double s_mu[DMAX], s_ls[DMAX], s_sg[DMAX];
  // t family, Philox: the row's samples x, [DMAX][256] (see below), and the row's
  // log-q constant sum_d (t_const - log sigma_d) (the same for every row of the block)
  __shared__ double s_x[(TFAM && !HOST) ? DMAX * 256 : 1];
  __shared__ double s_lqc;
  // row q of a batched launch (vb_log_weights_rows): its own lambda, output
  // row, noise rows and Philox stream (stream + q * stride)
  const int q = blockIdx.y;
  lam += (long long)q * 2 * D;
  lw += (long long)q * m;
  if (xs) xs += (long long)q * m * D;
  if (noise) noise += (long long)q * m * D;
  rng.stream += (uint32_t)q * stride;
  // the block's lambda row and sigma = exp(log sigma) once per block (the same
  // bits as per draw), with the Box-Muller tables
  if ((int)threadIdx.x < D) {
    const double ls = lam[D + threadIdx.x];
    s_mu[threadIdx.x] = lam[threadIdx.x];
    s_ls[threadIdx.x] = ls;
    s_sg[threadIdx.x] = exp(ls);
  }
  if constexpr (!HOST) load_bm_tables(s_sct, s_lt);
  __syncthreads();
  if constexpr (TFAM && !HOST) {
    if (threadIdx.x == 0) {   // (d ascending: the order the rows once summed it in)
      double c = 0.0;
      for (int d = 0; d < D; ++d) c += t_const - s_ls[d];
      s_lqc = c;
    }
    __syncthreads();
  }
  const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
  if (r >= m) return;
  double x[DMAX], g[DMAX];
  double lq = 0.0;
  if constexpr (TFAM && !HOST) {
    // Bailey t draws (the log-weight draws of the t family, bailey_t; vbrng.c
    // family 2), log q = t_const - (df + 1)/2 log1p(T^2 / df) - log sigma at the
    // draw itself (x = mu + sigma T rounded moves it by ~1e-16 relative).  One
    // column pair per iteration of a rolled loop (the polynomial constants stay in
    // registers; unrolled, they were re-made for every variate), x written to LDS,
    // then read back as a register array for the target.
    // The row's log1p(T_d^2 / df) terms as ONE log of the product of the (1 + T_d^2 /
    // df), its binary exponent split off after every pair (a factor reaches 2^(82 / df)
    // for U1 = 2^-41: small df would overflow a plain product).  The product's ~D
    // roundings move the log by ~D ulp of its magnitude -- ~1e-15 absolute against the
    // oracle's sum of log1p (vbrng.c family 2; tests/test_gpu_bailey.py at 1e-12).  Nine
    // of ten table log1p per row at D = 10 become multiplies (round 6, config 5's bounds
    // stage).
    const double c2 = -2.0 / df, hdf1 = 0.5 * (df + 1.0);
    const int t = threadIdx.x;
    double pr = 1.0;
    int pe = 0;
#pragma unroll 1
    for (int j = 0; 2 * j < D; ++j) {
      const u4 w = rng.draw((uint32_t)j, (uint32_t)r, step, kBaileyPurpose);
      double ya, yb;
      const double ta = bailey_t_y(w.x, w.z, df, c2, s_sct, s_lt, ya);
      const double tb = bailey_t_y(w.y, w.w, df, c2, s_sct, s_lt, yb);
      const int d = 2 * j;
      const double xa = ta * s_sg[d] + s_mu[d];
      pr = fma(pr, ya, pr);
      s_x[d * 256 + t] = xa;
      if (d + 1 < D) {
        const double xb = tb * s_sg[d + 1] + s_mu[d + 1];
        pr = fma(pr, yb, pr);
        s_x[(d + 1) * 256 + t] = xb;
        if (xs) xs[r * D + d + 1] = xb;
      }
      if (xs) xs[r * D + d] = xa;
      int e;
      pr = frexp(pr, &e);
      pe += e;
    }
    const double dpe = (double)pe;
    lq = s_lqc - hdf1 * fma(dpe, 0.6931471805598903, fma(dpe, 5.497923018708371e-14, log_unit_tab(pr, s_lt)));
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      x[d] = d < D ? s_x[d * 256 + t] : 0.0;
      g[d] = 0.0;
    }
  } else {
#pragma unroll
    for (int j = 0; j < (DMAX + 1) / 2; ++j) {
      double e0 = 0.0, e1 = 0.0;
      if (2 * j < D)
        draw_pair<TFAM, HOST>(rng, noise, D, r, j, step, t_scale, shape, e0, e1, s_sct, s_lt);
      const double e[2] = {e0, e1};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int d = 2 * j + c;
        if (d >= DMAX) continue;
        x[d] = 0.0;
        g[d] = 0.0;
        if (d < D) {
          const double mu = s_mu[d], sg = s_sg[d];
          x[d] = e[c] * sg + mu;
          lq += logq1s<TFAM, HOST>(x[d], mu, s_ls[d], sg, df, t_const, s_lt);
          if (xs) xs[r * D + d] = x[d];
        }
      }
    }
  }
  double lp;
  if constexpr (std::is_same_v<TGT, EightSchools> && !HOST) {
    lp = TGT::template lp_tab<DMAX>(x, D, s_lt);
    (void)g;
  } else {
    lp = RowOf<TGT>::template row<DMAX>(x, g, D);
  }
  lw[r] = lp - lq;
}

// -------------------------------------------------------------------------
// launchers
// -------------------------------------------------------------------------
bool target_separable(int tgt) { return tgt == 0 || tgt == 1; }

// Split of the column pairs between multi-pair (PPW_BIG) and 1-pair waves: below
// 8 192 pairs one 4-pair wave per SIMD (1 024 of them), then 1-pair waves -- measured
// fastest at D = 1e4 (profiles/r01/ab_layouts_q.json; round 5: two 2-pair waves + 1-pair
// waves per SIMD 87 us, all 2-pair 97, all 1-pair 104, a 4-pair wave on every SIMD
// 75.0, against 75.1 us for this split, profiles/r05/headline_layout*.log); larger D
// generalises it (see the second branch).  Blocks of big waves come first so
// round-robin dispatch deals the same mix to every CU.
static void sep_split(SepArgs& a) {
  constexpr int big = 4;
  const int np = a.n_pairs;
  int pairs2;
  if (np < 2 * 4096) {
    pairs2 = np > 4096 + 1024 ? 4096 : (np > 1024 ? np - 1024 : 0);
  } else {
    // larger D: L layers of one 4-pair wave per SIMD and the rest in 1-pair
    // waves while that stays within ~4 resident waves per SIMD; beyond, all
    // 4-pair waves (their fixed per-step cost per pair is ~4x lower:
    // profiles/r01_sweep_layouts.json)
    const int layers = np / 4096, rest = np - 4096 * layers;
    pairs2 = layers + (rest + 1023) / 1024 <= 4 ? 4096 * layers : np;
  }
  pairs2 -= pairs2 % (4 * big);   // whole blocks of 4 big waves
  a.pairs2 = pairs2;
  a.blocks2 = pairs2 / (4 * big);
  const int rest = np - pairs2;
  a.blocks1 = (rest + 3) / 4;
}

template <class TGT, bool TFAM, bool HOST, bool REG>
static void sep_launch(const SepArgs& a, hipStream_t s) {
  // the optimisation launches (no emitted gradient, plain KLVI value) take the
  // instance with those flags compiled in (sep_kernel's ADV)
  if (!a.emit_grad && a.pd == 0)
    hipLaunchKernelGGL((sep_kernel<TGT, TFAM, HOST, 4, REG, true>), dim3(a.blocks2 + a.blocks1),
                       dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((sep_kernel<TGT, TFAM, HOST, 4, REG>), dim3(a.blocks2 + a.blocks1), dim3(256),
                       0, s, a);
}

template <class TGT>
static hipError_t sep_dispatch(int fam, bool host, SepArgs a, hipStream_t s) {
  sep_split(a);
  const bool reg = a.W <= 16 || a.emit_grad;
  if (host) {
    // host noise holds standardized draws for either family
    if (reg) sep_launch<TGT, false, true, true>(a, s);
    else sep_launch<TGT, false, true, false>(a, s);
  } else if (fam == 1) {
    if (reg) sep_launch<TGT, true, false, true>(a, s);
    else sep_launch<TGT, true, false, false>(a, s);
  } else {
    if (reg) sep_launch<TGT, false, false, true>(a, s);
    else sep_launch<TGT, false, false, false>(a, s);
  }
  return hipGetLastError();
}

hipError_t launch_sep(int fam, int tgt, bool host, const SepArgs& a, hipStream_t s) {
  switch (tgt) {
    case 0: return sep_dispatch<IsoGauss>(fam, host, a, s);
    case 1: return sep_dispatch<Mixture>(fam, host, a, s);
    default: return hipErrorInvalidValue;
  }
}

bool block_pf_layout(int N, int D, bool need_lq, int pf_mode) {
  return N >= 1 && D >= 1 && D <= kBlockDMax && block_layout(N, D, true, need_lq, pf_mode).pf;
}

// Threads per problem: the draws of one step spread over ceil(N/64) waves (<= 4).
// Threads per problem: host noise -> one thread per sample (<= 4 waves); Philox ->
// enough waves for the (sample, pair) draw items of a step (<= 8 waves).
inline unsigned block_threads(const BlockArgs& a, bool host) {
  return (unsigned)block_layout(a.N, a.D, host, a.chivi || a.pd, host ? a.pf : 0).nt;
}

template <class TGT, int DM>
static hipError_t block_dispatch_dm(int fam, bool host, const BlockArgs& a, int nprob,
                                    hipStream_t s) {
  const dim3 grid(nprob), block(block_threads(a, host));
  const BlockLayout L = block_layout(a.N, a.D, true, a.chivi || a.pd, a.pf);
  const bool pf = host && L.pf;
  if constexpr (DM <= kBlockSplitMaxD) {
    if (host && L.split) {
      // the benchmark modes with their flags compiled in (block_kernel's HOT)
      const bool chivi_hot = a.noise_lq && a.W >= 1 && a.W <= kBlockQpreMaxW;
      const int hot = (!a.emit_grad && a.opt == 0 && !a.pd) ? (a.chivi ? (chivi_hot ? 2 : 0) : 1) : 0;
#define VB_SPLIT_LAUNCH(F, H) \
  hipLaunchKernelGGL((block_kernel<TGT, F, true, DM, true, true, H>), grid, block, 0, s, a)
      if (fam == 1) {
        if (hot == 1) VB_SPLIT_LAUNCH(true, 1);
        else if (hot == 2) VB_SPLIT_LAUNCH(true, 2);
        else VB_SPLIT_LAUNCH(true, 0);
      } else {
        if (hot == 1) VB_SPLIT_LAUNCH(false, 1);
        else if (hot == 2) VB_SPLIT_LAUNCH(false, 2);
        else VB_SPLIT_LAUNCH(false, 0);
      }
#undef VB_SPLIT_LAUNCH
      return hipGetLastError();
    }
  }
  if (host && fam == 1) {
    if (pf)
      hipLaunchKernelGGL((block_kernel<TGT, true, true, DM, true>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((block_kernel<TGT, true, true, DM>), grid, block, 0, s, a);
  } else if (host) {
    if (pf)
      hipLaunchKernelGGL((block_kernel<TGT, false, true, DM, true>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((block_kernel<TGT, false, true, DM>), grid, block, 0, s, a);
  } else if (fam == 1) {
    // (runs pre-draw the t family's Philox noise by default: launch_block_predraw)
    hipLaunchKernelGGL((block_kernel<TGT, true, false, DM>), grid, block, 0, s, a);
  } else {
    hipLaunchKernelGGL((block_kernel<TGT, false, false, DM>), grid, block, 0, s, a);
  }
  return hipGetLastError();
}

// Register arrays are sized by DMAX: pick the smallest instantiation >= D.
template <class TGT>
static hipError_t block_dispatch(int fam, bool host, const BlockArgs& a, int nprob,
                                 hipStream_t s) {
  if constexpr (std::is_same_v<TGT, EightSchools>) {
    return block_dispatch_dm<TGT, 10>(fam, host, a, nprob, s);
  } else {
    if (a.D <= 2) return block_dispatch_dm<TGT, 2>(fam, host, a, nprob, s);
    if (a.D <= 4) return block_dispatch_dm<TGT, 4>(fam, host, a, nprob, s);
    if (a.D <= 10) return block_dispatch_dm<TGT, 10>(fam, host, a, nprob, s);
    return block_dispatch_dm<TGT, kBlockDMax>(fam, host, a, nprob, s);
  }
}

// In host-noise mode the t family's CHIVI log q still needs df: the kernel reads
// a.df / a.t_const, which the caller fills for fam == 1.  The TFAM template flag
// only selects the in-kernel t sampler, so for host noise we must pick the log q
// form from the family at run time: handled by routing t-family CHIVI through the
// TFAM=true instantiation with HOST=true.
template <class TGT>
static hipError_t block_dispatch_full(int fam, bool host, const BlockArgs& a, int nprob,
                                      hipStream_t s) {
  return block_dispatch<TGT>(fam, host, a, nprob, s);
}

hipError_t launch_block(int fam, int tgt, bool host, const BlockArgs& a, int nprob,
                        hipStream_t s) {
  switch (tgt) {
    case 0: return block_dispatch_full<IsoGauss>(fam, host, a, nprob, s);
    case 1: return block_dispatch_full<Mixture>(fam, host, a, nprob, s);
    case 2: return block_dispatch_full<Funnel>(fam, host, a, nprob, s);
    case 3: return block_dispatch_full<EightSchools>(fam, host, a, nprob, s);
    default: return hipErrorInvalidValue;
  }
}

#ifdef VB_SEP_TS
extern "C" int vb_debug_sep_ts(unsigned long long* out, int n_waves) {
  if (n_waves > kTsWaves) n_waves = kTsWaves;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sep_ts),
                                    sizeof(unsigned long long) * 16 * n_waves, 0,
                                    hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    e = hipMemcpyFromSymbol(out + 16 * n_waves, HIP_SYMBOL(g_sep_clk),
                            sizeof(unsigned long long) * 16 * n_waves, 0, hipMemcpyDeviceToHost);
  return (int)e;
}
#endif

hipError_t launch_sep_values(const double* vpart, int n_steps, int n_waves, double c0,
                             double* values, hipStream_t s) {
  hipLaunchKernelGGL(sep_values_kernel, dim3(n_steps), dim3(kValThreads), 0, s, vpart, n_waves,
                     c0, values);
  return hipGetLastError();
}

hipError_t launch_row_mean(const double* hist, long long rows, long long P, long long nprob,
                           double* out, hipStream_t s) {
  const long long tot = P * nprob;
  hipLaunchKernelGGL(row_mean_kernel, dim3((unsigned)((tot + kRowMeanThreads - 1) / kRowMeanThreads)),
                     dim3(kRowMeanThreads), 0, s, hist, rows, P, nprob, out);
  return hipGetLastError();
}

hipError_t launch_sample(int fam, int D, long long n, const double* lam, double t_scale,
                         double shape, const double* noise, uint32_t k0, uint32_t k1,
                         uint32_t stream, uint32_t step, double* x, hipStream_t s) {
  const long long tot = n * ((D + 1) / 2);
  if (tot == 0) return hipSuccess;
  const dim3 grid((unsigned)((tot + 255) / 256)), block(256);
  const Rng rng{k0, k1, stream};
  if (noise)
    hipLaunchKernelGGL((sample_kernel<false, true>), grid, block, 0, s, D, n, lam, t_scale, shape,
                       noise, rng, step, x);
  else if (fam == 1)
    hipLaunchKernelGGL((sample_kernel<true, false>), grid, block, 0, s, D, n, lam, t_scale, shape,
                       noise, rng, step, x);
  else
    hipLaunchKernelGGL((sample_kernel<false, false>), grid, block, 0, s, D, n, lam, t_scale,
                       shape, noise, rng, step, x);
  return hipGetLastError();
}

// Bailey t samples x [m][D] of a mean-field t family (the log-weight draws of the
// materialised path), one thread per (row, column pair) as sample_kernel
__global__ __launch_bounds__(256) void sample_bailey_kernel(int D, long long n, const double* lam,
                                                            double df, Rng rng, uint32_t step,
                                                            double* x) {
  __shared__ double2 s_sct[kSinCosN];
  __shared__ double2 s_lt[kLogN + kLogU01N];
  load_bm_tables(s_sct, s_lt);
  __syncthreads();
  const int npairs = (D + 1) / 2;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= n * npairs) return;
  const long long r = idx / npairs;
  const int j = (int)(idx % npairs);
  const u4 w = rng.draw((uint32_t)j, (uint32_t)r, step, kBaileyPurpose);
  const double c2 = -2.0 / df;
  double l1;
  const double ta = bailey_t(w.x, w.z, df, c2, s_sct, s_lt, l1);
  const double tb = bailey_t(w.y, w.w, df, c2, s_sct, s_lt, l1);
  x[r * D + 2 * j] = ta * exp(lam[D + 2 * j]) + lam[2 * j];
  if (2 * j + 1 < D) x[r * D + 2 * j + 1] = tb * exp(lam[D + 2 * j + 1]) + lam[2 * j + 1];
}

hipError_t launch_sample_bailey(int D, long long m, const double* lam, double df, uint32_t k0,
                                uint32_t k1, uint32_t stream, uint32_t step, double* x,
                                hipStream_t s) {
  const long long tot = m * ((D + 1) / 2);
  if (tot == 0) return hipSuccess;
  const Rng rng{k0, k1, stream};
  hipLaunchKernelGGL(sample_bailey_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, D,
                     m, lam, df, rng, step, x);
  return hipGetLastError();
}

// Fused materialised step for separable targets on wide rows.  Thread t of
// block (c, b) owns column pair j = 256 c + t and walks kRowsPerBlock rows
// b kRowsPerBlock + q: it draws the pair (same Philox counters as
// sample_kernel, table transcendentals as the fused KLVI kernels), forms
// x = eps sigma + mu, evaluates the target log density and its gradient and
// (CHIVI / klvi_pd) the family log density of the same x, all from registers:
// one pass over the rows instead of three kernels that re-read x from HBM.
// The column constants (mu, sigma, 1/sigma, log q offsets) load once per
// thread.  Writes x, grad and the chunk partials logp[c n + r], logq[c n + r]
// (with_lq); the consumer sums the mfw_rows_parts(D) partials of a row in
// chunk order (deterministic).
// log1p of the t family's log q term: LDS-table form when the Box-Muller tables
// are loaded (Philox draws), the library log1p otherwise.
template <bool HOST>
__device__ __forceinline__ double lq1p(double y, const double2* ltab) {
#ifdef VB_NO_LQ_TAB
  return log1p(y);
#else
  if constexpr (HOST) return log1p(y);
  else return log1p_pos_tab(y, ltab);
#endif
}

constexpr int kRowChunkPairs = 256;
constexpr int kRowsPerBlock = 4;  // 1, 2, 8: within 3 % (D = 1e4, N = 128)

int mfw_rows_parts(int D) { return ((D + 1) / 2 + kRowChunkPairs - 1) / kRowChunkPairs; }

template <class TGT, bool TFAM, bool HOST>
__global__ __launch_bounds__(256) void mfw_rows_kernel(int D, long long n, const double* lam,
                                                       double t_scale, double shape, double df,
                                                       double t_const, int with_lq,
                                                       const double* noise, Rng rng, uint32_t step,
                                                       double* x, double* grad, double* logp,
                                                       double* logq) {
  __shared__ double2 s_sct[HOST ? 1 : kSinCosN];
  __shared__ double2 s_lt[HOST ? 1 : kLogN + kLogU01N];
  __shared__ double red[2][kRowsPerBlock][4];
  if constexpr (!HOST) {
    load_bm_tables(s_sct, s_lt);
    __syncthreads();
  }
  const int c = blockIdx.x;
  const int j = c * kRowChunkPairs + (int)threadIdx.x;
  const int npairs = (D + 1) / 2;
  const bool act = j < npairs;
  const int dA = 2 * j, dB = 2 * j + 1;
  const bool hasB = act && dB < D;
  const bool evenD = (D & 1) == 0;
  double muA = 0.0, sA = 1.0, isA = 1.0, cA = 0.0;
  double muB = 0.0, sB = 1.0, isB = 1.0, cB = 0.0;
  if (act) {
    const double ls = lam[D + dA];
    muA = lam[dA];
    sA = exp(ls);
    isA = 1.0 / sA;
    cA = TFAM ? t_const - ls : -ls - 0.5 * kLog2Pi;
  }
  if (hasB) {
    const double ls = lam[D + dB];
    muB = lam[dB];
    sB = exp(ls);
    isB = 1.0 / sB;
    cB = TFAM ? t_const - ls : -ls - 0.5 * kLog2Pi;
  }
  const double hexp = 0.5 * (df + 1.0), idf = 1.0 / df;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long r0 = (long long)blockIdx.y * kRowsPerBlock;
#pragma unroll 1
  for (int q = 0; q < kRowsPerBlock; ++q) {
    const long long r = r0 + q;
    double lp = 0.0, lq = 0.0;
    if (act && r < n) {
      double eA, eB;
      if constexpr (HOST) {
        eA = noise[r * D + dA];
        eB = hasB ? noise[r * D + dB] : 0.0;
      } else {
        normal_pair_tab(rng.draw((uint32_t)j, (uint32_t)r, step, 0u), eA, eB, s_sct, s_lt);
        if constexpr (TFAM) {
          double ga, gb;
          gamma_pair<true>(rng, (uint32_t)j, (uint32_t)r, step, shape, ga, gb, s_sct, s_lt);
          eA = t_scale * eA / sqrt(ga);
          eB = t_scale * eB / sqrt(gb);
        }
      }
      double gA, gB = 0.0;
      const double xA = eA * sA + muA, xB = eB * sB + muB;
      lp = TGT::lp1(xA, gA);
      const double zA = (xA - muA) * isA;
      lq = TFAM ? cA - lq1p<HOST>(zA * zA * idf, s_lt) * hexp : fma(-0.5 * zA, zA, cA);
      if (hasB) {
        lp += TGT::lp1(xB, gB);
        const double zB = (xB - muB) * isB;
        lq += TFAM ? cB - lq1p<HOST>(zB * zB * idf, s_lt) * hexp : fma(-0.5 * zB, zB, cB);
      }
      if (evenD) {  // 16-byte stores: the wave writes 1 KB of x and of grad contiguously
        *reinterpret_cast<double2*>(x + r * D + dA) = double2{xA, xB};
        *reinterpret_cast<double2*>(grad + r * D + dA) = double2{gA, gB};
      } else {
        x[r * D + dA] = xA;
        grad[r * D + dA] = gA;
        if (hasB) {
          x[r * D + dB] = xB;
          grad[r * D + dB] = gB;
        }
      }
    }
    lp = wave_sum_dpp(lp);
    if (with_lq) lq = wave_sum_dpp(lq);
    if (lane == 0) {
      red[0][q][wave] = lp;
      red[1][q][wave] = lq;
    }
  }
  __syncthreads();
  if (threadIdx.x < kRowsPerBlock) {
    const int q = threadIdx.x;
    const long long r = r0 + q;
    if (r < n) {
      logp[(long long)c * n + r] = (red[0][q][0] + red[0][q][1]) + (red[0][q][2] + red[0][q][3]);
      if (with_lq)
        logq[(long long)c * n + r] = (red[1][q][0] + red[1][q][1]) + (red[1][q][2] + red[1][q][3]);
    }
  }
}

template <class TGT>
static void mfw_rows_dispatch(int fam, int D, long long n, const double* lam, double t_scale,
                              double shape, double df, double t_const, bool with_lq,
                              const double* noise, const Rng& rng, uint32_t step, double* x,
                              double* grad, double* logp, double* logq, hipStream_t s) {
  const dim3 g((unsigned)mfw_rows_parts(D), (unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock)),
      b(256);
  const int wl = with_lq ? 1 : 0;
  if (noise && fam == 1)
    hipLaunchKernelGGL((mfw_rows_kernel<TGT, true, true>), g, b, 0, s, D, n, lam, t_scale, shape,
                       df, t_const, wl, noise, rng, step, x, grad, logp, logq);
  else if (noise)
    hipLaunchKernelGGL((mfw_rows_kernel<TGT, false, true>), g, b, 0, s, D, n, lam, t_scale, shape,
                       df, t_const, wl, noise, rng, step, x, grad, logp, logq);
  else if (fam == 1)
    hipLaunchKernelGGL((mfw_rows_kernel<TGT, true, false>), g, b, 0, s, D, n, lam, t_scale, shape,
                       df, t_const, wl, noise, rng, step, x, grad, logp, logq);
  else
    hipLaunchKernelGGL((mfw_rows_kernel<TGT, false, false>), g, b, 0, s, D, n, lam, t_scale, shape,
                       df, t_const, wl, noise, rng, step, x, grad, logp, logq);
}

bool mfw_rows_fusable(int tgt, int D, long long n) {
  return (tgt == 0 || tgt == 1) && D >= kWideRowD && n >= 1 && n <= 65535;
}

hipError_t launch_mfw_rows(int fam, int tgt, int D, long long n, const double* lam, double t_scale,
                           double shape, double df, double t_const, bool with_lq,
                           const double* noise, uint32_t k0, uint32_t k1, uint32_t stream,
                           uint32_t step, double* x, double* grad, double* logp, double* logq,
                           hipStream_t s) {
  if (!mfw_rows_fusable(tgt, D, n)) return hipErrorInvalidValue;
  const Rng rng{k0, k1, stream};
  if (tgt == 0)
    mfw_rows_dispatch<IsoGauss>(fam, D, n, lam, t_scale, shape, df, t_const, with_lq, noise, rng,
                                step, x, grad, logp, logq, s);
  else
    mfw_rows_dispatch<Mixture>(fam, D, n, lam, t_scale, shape, df, t_const, with_lq, noise, rng,
                               step, x, grad, logp, logq, s);
  return hipGetLastError();
}

hipError_t launch_family_logdensity(int fam, int D, long long n, const double* lam, double df,
                                    double t_const, const double* x, double* out,
                                    hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (D >= kWideRowD && n <= 65535) {
    if (fam == 1)
      hipLaunchKernelGGL((family_logdensity_rowblock_kernel<true>), dim3((unsigned)n), dim3(1024),
                         0, s, D, lam, df, t_const, x, out);
    else
      hipLaunchKernelGGL((family_logdensity_rowblock_kernel<false>), dim3((unsigned)n), dim3(1024),
                         0, s, D, lam, df, t_const, x, out);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
  if (fam == 1)
    hipLaunchKernelGGL((family_logdensity_kernel<true>), grid, block, 0, s, D, n, lam, df,
                       t_const, x, out);
  else
    hipLaunchKernelGGL((family_logdensity_kernel<false>), grid, block, 0, s, D, n, lam, df,
                       t_const, x, out);
  return hipGetLastError();
}

hipError_t launch_target_logdensity(int tgt, int D, long long n, const double* x, double* out,
                                    double* grad, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const dim3 gw((unsigned)((n + 3) / 4)), gt((unsigned)((n + 255) / 256)), block(256);
  if (D >= kWideRowD && n <= 65535 && tgt <= 2) {
    const dim3 gb((unsigned)n), bb(1024);
    switch (tgt) {
      case 0: hipLaunchKernelGGL((target_sep_rowblock_kernel<IsoGauss>), gb, bb, 0, s, D, x, out, grad); break;
      case 1: hipLaunchKernelGGL((target_sep_rowblock_kernel<Mixture>), gb, bb, 0, s, D, x, out, grad); break;
      default: hipLaunchKernelGGL(funnel_rowblock_kernel, gb, bb, 0, s, D, x, out, grad); break;
    }
    return hipGetLastError();
  }
  switch (tgt) {
    case 0: hipLaunchKernelGGL((target_sep_kernel<IsoGauss>), gw, block, 0, s, D, n, x, out, grad); break;
    case 1: hipLaunchKernelGGL((target_sep_kernel<Mixture>), gw, block, 0, s, D, n, x, out, grad); break;
    case 2:
      if (D <= kBlockDMax)
        hipLaunchKernelGGL((target_row_kernel<Funnel, kBlockDMax>), gt, block, 0, s, D, n, x, out,
                           grad);
      else
        hipLaunchKernelGGL(funnel_wide_kernel, gw, block, 0, s, D, n, x, out, grad);
      break;
    case 3:
      hipLaunchKernelGGL((target_row_kernel<EightSchools, kBlockDMax>), gt, block, 0, s, D, n, x,
                         out, grad);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <class TGT, bool TFAM, bool HOST>
static void logw_launch(int D, long long m, const double* lam, double t_scale, double shape,
                        double df, double t_const, const double* noise, Rng rng, uint32_t step,
                        int rows, uint32_t stride, double* lw, double* xs, hipStream_t s) {
  if constexpr (TGT::kSeparable) {
    if (D > kBlockDMax) {
      hipLaunchKernelGGL((logw_sep_kernel<TGT, TFAM, HOST>),
                         dim3((unsigned)((m + 3) / 4), (unsigned)rows), dim3(256), 0, s, D, m,
                         lam, t_scale, shape, df, t_const, noise, rng, step, stride, lw, xs);
      return;
    }
  }
  {
    // register arrays sized by the smallest instance >= D (as block_dispatch)
    const dim3 g((unsigned)((m + 255) / 256), (unsigned)rows);
#define VB_LOGW(DM)                                                                            \
  hipLaunchKernelGGL((logw_row_kernel<TGT, TFAM, HOST, DM>), g, dim3(256), 0, s, D, m, lam,   \
                     t_scale, shape, df, t_const, noise, rng, step, stride, lw, xs)
    if (D <= 2) VB_LOGW(2);
    else if (D <= 4) VB_LOGW(4);
    else if (D <= 10) VB_LOGW(10);
    else VB_LOGW(kBlockDMax);
#undef VB_LOGW
  }
}

template <class TGT>
static void logw_fam(int fam, bool host, int D, long long m, const double* lam, double t_scale,
                     double shape, double df, double t_const, const double* noise, Rng rng,
                     uint32_t step, int rows, uint32_t stride, double* lw, double* xs,
                     hipStream_t s) {
  if (fam == 1) {
    if (host) logw_launch<TGT, true, true>(D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s);
    else logw_launch<TGT, true, false>(D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s);
  } else {
    if (host) logw_launch<TGT, false, true>(D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s);
    else logw_launch<TGT, false, false>(D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s);
  }
}

hipError_t launch_log_weights(int fam, int tgt, int D, long long m, const double* lam,
                              double t_scale, double shape, double df, double t_const,
                              const double* noise, uint32_t k0, uint32_t k1, uint32_t stream,
                              uint32_t step, double* lw, double* xs, hipStream_t s, int rows,
                              uint32_t stride) {
  if (m == 0 || rows <= 0) return hipSuccess;
  const Rng rng{k0, k1, stream};
  const bool host = noise != nullptr;
  switch (tgt) {
    case 0: logw_fam<IsoGauss>(fam, host, D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s); break;
    case 1: logw_fam<Mixture>(fam, host, D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s); break;
    case 2: logw_fam<Funnel>(fam, host, D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s); break;
    case 3: logw_fam<EightSchools>(fam, host, D, m, lam, t_scale, shape, df, t_const, noise, rng, step, rows, stride, lw, xs, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_adagrad_update(long long P, double* lam, const double* g, double* ring, int W,
                                 long long step, double lr, double eps, const double* scale,
                                 hipStream_t s, double* hrow) {
  hipLaunchKernelGGL(adagrad_update_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P,
                     lam, g, ring, W, step, lr, eps, scale, hrow);
  return hipGetLastError();
}

hipError_t launch_ia_update(int opt, long long P, double* lam, const double* g, double* state,
                            long long step, double lr, double eps, double norm2,
                            double* old_out, hipStream_t s) {
  hipLaunchKernelGGL(ia_update_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, opt, P,
                     lam, g, state, step, lr, eps, norm2, old_out);
  return hipGetLastError();
}

}  // namespace vbk

// vb_device.hpp — device building blocks shared by the gfx950 kernels.
//
//  * Philox4x32-10 counter RNG (Salmon et al., SC'11), counter layout
//      c0 = column pair j, c1 = sample n, c2 = step, c3 = stream | purpose<<24
//    key = (seed lo, seed hi).  Purpose 0 = standard-normal pairs, purpose
//    1+k = k-th Marsaglia-Tsang gamma proposal.  The layout makes every draw
//    addressable, so kernels regenerate noise instead of storing it, and any
//    tiling of (n, d) produces the same draws.
//  * normal pair: Box-Muller on two 52-bit uniforms (u1 in (0,1), u2 in [0,1)).
//  * t draws follow numpy's legacy standard_t structure
//    sqrt(df/2) * gauss / sqrt(gamma(df/2)) (numpy legacy distributions.c),
//    with gamma by Marsaglia-Tsang (shape >= 1, which df > 2 guarantees).
//  * target log densities with gradients.
//
// Everything is fp64; the build never uses fast-math (PSIS needs IEEE inf).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vb_tables.hpp"

namespace vbd {

constexpr double kLog2Pi = 1.8378770664093454835606594728112;  // log(2*pi)
constexpr double kLn2 = 0.69314718055994530941723212145818;

struct u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                     uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    // three-input XOR in one v_bitop3_b32 (gfx950, truth table 0x96)
    const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
    const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return u4{c0, c1, c2, c3};
}

struct Rng {
  uint32_t k0, k1;      // key
  uint32_t stream;      // 24-bit stream id (restart / family instance)
  __device__ __forceinline__ u4 draw(uint32_t pair, uint32_t sample, uint32_t step,
                                     uint32_t purpose) const {
    return philox(pair, sample, step, (stream & 0x00FFFFFFu) | (purpose << 24), k0, k1);
  }
};

// ---- fp64 transcendentals for noise generation --------------------------------
// Box-Muller needs log, sqrt and sin/cos of uniforms only.  These short forms
// (about 1 ulp) replace the general ocml routines (which carry extra-precision
// arithmetic and special-case handling the noise path never needs): the
// transform is ~40% cheaper.  The C oracle uses libm; tests compare at 1e-14.

// Horner step a * b + c as a three-address VOP3 v_fma_f64.  Left to itself the
// compiler emits v_mov_b64 (copy of the loop-invariant coefficient c) + v_fmac,
// two instructions per step, because fmac's accumulator is also its destination.
__device__ __forceinline__ double hfma(double a, double b, double c) {
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// log(u) for u in (0, 1]: u = m 2^e with m in [sqrt(1/2), sqrt(2)),
// log m = 2 atanh(f) = 2 f sum_k f^2k / (2k+1), f = (m-1)/(m+1), |f| <= 0.1716.
__device__ __forceinline__ double log_unit(double u) {
  int e;
  double m = frexp(u, &e);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  const double num = m - 1.0, den = m + 1.0;
  double r = __builtin_amdgcn_rcp(den);
  r = fma(r, fma(-den, r, 1.0), r);
  r = fma(r, fma(-den, r, 1.0), r);
  double f = num * r;
  f = fma(r, fma(-den, f, num), f);
  const double f2 = f * f;
  double p = 0.04347826086956522;            // 1/23
  p = hfma(p, f2, 0.047619047619047616);      // 1/21
  p = hfma(p, f2, 0.05263157894736842);
  p = hfma(p, f2, 0.058823529411764705);
  p = hfma(p, f2, 0.06666666666666667);
  p = hfma(p, f2, 0.07692307692307693);
  p = hfma(p, f2, 0.09090909090909091);
  p = hfma(p, f2, 0.1111111111111111);
  p = hfma(p, f2, 0.14285714285714285);
  p = hfma(p, f2, 0.2);
  p = hfma(p, f2, 0.3333333333333333);
  const double de = (double)e;
  // ln2 = LN2_HI + LN2_LO, LN2_HI with trailing zero bits so de * LN2_HI is exact
  const double t = fma(2.0 * f * f2, p, 2.0 * f);
  return fma(de, 0.6931471805598903, fma(de, 5.497923018708371e-14, t));
}

// exp(x), ~1 ulp (max 1.07 ulp over 2e7 arguments against a long-double exp; the
// library form is also ~1 ulp): x = k ln2 + r, |r| <= ln2 / 2, exp(r) = 1 + r +
// r^2 q(r), q of degree 9 fitted on [-ln2/2, ln2/2] (scripts/gen_exp_coef.py), its
// Horner steps as three-address fmas -- the library's copy each coefficient into a
// register before a two-address fmac, ~31 instructions against ~23 here.  Overflow
// gives inf, underflow 0 (the argument clamped to [-746, 710] first), NaN stays NaN.
// Used on the serial chains of the block and column-pair kernels (the updated
// sigma = exp(log sigma), the targets' exp, the CHIVI rescale factors).
__device__ __forceinline__ double exp_fast(double x) {
  const double xc = fmin(fmax(x, -746.0), 710.0);
  const double k = rint(xc * 1.4426950408889634);
  double r = fma(-k, 6.93147180369123816490e-01, xc);   // ln2 high part: k ln2_hi exact
  r = fma(-k, 1.90821492927058770002e-10, r);
  double q = 2.5105102509207056e-08;
  q = hfma(q, r, 2.7620092546932737e-07);
  q = hfma(q, r, 2.755725563278083e-06);
  q = hfma(q, r, 2.4801521277219366e-05);
  q = hfma(q, r, 0.00019841269874702037);
  q = hfma(q, r, 0.0013888888917237376);
  q = hfma(q, r, 0.008333333333326141);
  q = hfma(q, r, 0.041666666666624025);
  q = hfma(q, r, 0.1666666666666667);
  q = hfma(q, r, 0.5000000000000001);
  const double e = fma(r * r, q, r) + 1.0;
  const double res = ldexp(e, (int)k);
  return x != x ? x : res;
}

// expm1(x) for 0 <= x <= 700, ~1 ulp: exp_fast's reduction x = k ln2 + r and its
// polynomial, expm1(r) = r + r^2 q(r) (no cancellation near 0), then
// 2^k (1 + expm1(r)) - 1 = 2^k expm1(r) + (2^k - 1) in one fma (2^k - 1 exact for
// k <= 53; larger k round it as 2^k, well within an ulp of the result).  The
// Bailey draws pass -(2/df) log U1 <= 57 / df.
__device__ __forceinline__ double expm1_pos(double x) {
  const double xc = x;
  const double k = rint(xc * 1.4426950408889634);
  double r = fma(-k, 6.93147180369123816490e-01, xc);
  r = fma(-k, 1.90821492927058770002e-10, r);
  double q = 2.5105102509207056e-08;
  q = hfma(q, r, 2.7620092546932737e-07);
  q = hfma(q, r, 2.755725563278083e-06);
  q = hfma(q, r, 2.4801521277219366e-05);
  q = hfma(q, r, 0.00019841269874702037);
  q = hfma(q, r, 0.0013888888917237376);
  q = hfma(q, r, 0.008333333333326141);
  q = hfma(q, r, 0.041666666666624025);
  q = hfma(q, r, 0.1666666666666667);
  q = hfma(q, r, 0.5000000000000001);
  const double p = fma(r * r, q, r);
  const double t = ldexp(1.0, (int)k);
  return fma(t, p, t - 1.0);
}

// log1p(w) for w >= 0 finite, without tables: log(1 + w) by log_unit (any positive
// normal argument) plus the rounding correction of 1 + w; ~1 ulp, ~35
// instructions against the library's double-double ~100
__device__ __forceinline__ double log1p_pos_fast(double w) {
  const double u = 1.0 + w;
  const double corr = (w - (u - 1.0)) * __builtin_amdgcn_rcp(u);
  return log_unit(u) + corr;
}

// sqrt(y) for y > 0 normal: rsq seed + Goldschmidt refinement.
__device__ __forceinline__ double sqrt_pos(double y) {
  const double r = __builtin_amdgcn_rsq(y);
  double h = 0.5 * r;
  double s = y * r;
  const double e = fma(-s, h, 0.5);
  s = fma(s, e, s);
  h = fma(h, e, h);
  const double d = fma(-s, s, y);
  return fma(d, h, s);
}

// sin(pi x), cos(pi x) for x in [0, 2]: octant reduction + Taylor on [-pi/4, pi/4].
__device__ __forceinline__ void sincospi_unit(double x, double& sn, double& cs) {
  const double q = rint(x + x);            // 0..4
  const double r = fma(-0.5, q, x);        // exact, |r| <= 1/4
  const double th = fma(r, 3.141592653589793, r * 1.2246467991473532e-16);
  const double t2 = th * th;
  double ps = -8.22063524662433e-18;
  ps = hfma(ps, t2, 2.8114572543455206e-15);
  ps = hfma(ps, t2, -7.647163731819816e-13);
  ps = hfma(ps, t2, 1.6059043836821613e-10);
  ps = hfma(ps, t2, -2.505210838544172e-08);
  ps = hfma(ps, t2, 2.7557319223985893e-06);
  ps = hfma(ps, t2, -0.0001984126984126984);
  ps = hfma(ps, t2, 0.008333333333333333);
  ps = hfma(ps, t2, -0.16666666666666666);
  const double s0 = fma(th * t2, ps, th);
  double pc = 4.110317623312165e-19;
  pc = hfma(pc, t2, -1.5619206968586225e-16);
  pc = hfma(pc, t2, 4.779477332387385e-14);
  pc = hfma(pc, t2, -1.1470745597729725e-11);
  pc = hfma(pc, t2, 2.08767569878681e-09);
  pc = hfma(pc, t2, -2.755731922398589e-07);
  pc = hfma(pc, t2, 2.48015873015873e-05);
  pc = hfma(pc, t2, -0.001388888888888889);
  pc = hfma(pc, t2, 0.041666666666666664);
  pc = hfma(pc, t2, -0.5);
  const double c0 = fma(t2, pc, 1.0);
  const int k = ((int)q) & 3;
  const double a = (k & 1) ? c0 : s0;     // |sin| or |cos| swapped on odd octant pairs
  const double b = (k & 1) ? s0 : c0;
  sn = (k & 2) ? -a : a;
  cs = (k == 1 || k == 2) ? -b : b;
}

// ---- table-driven forms (fused kernel; tables in LDS, vb_tables.hpp) ---------
// log(u), u in (0, 1]: u = m 2^e, m in [sqrt(1/2), sqrt(2)); c = 1 + i/64 the
// nearest table point, log m = -log(inv_c) + log1p(m inv_c - 1), |r| < 0.0113,
// log1p to r^9.  At m ~ 1 the entry is exactly (1, 0): no cancellation.
__device__ __forceinline__ double log_unit_tab(double u, const double2* ltab) {
  int e;
  double m = frexp(u, &e);
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  // exact: m in [0.5, 2); the clamp only matters for 0 / inf / NaN arguments,
  // which callers route to the general log (memory safety)
  const int i = min(max((int)rint(hfma(m, 64.0, -64.0)), kLogLo), kLogLo + kLogN - 1);
  const double2 t = ltab[i - kLogLo];
  const double r = fma(m, t.x, -1.0);
  double p = 0.1111111111111111;                 // 1/9
  p = hfma(p, r, -0.125);
  p = hfma(p, r, 0.14285714285714285);
  p = hfma(p, r, -0.16666666666666666);
  p = hfma(p, r, 0.2);
  p = hfma(p, r, -0.25);
  p = hfma(p, r, 0.3333333333333333);
  p = hfma(p, r, -0.5);
  const double l1p = fma(r * r, p, r);
  const double de = (double)e;
  return fma(de, 0.6931471805598903, fma(de, 5.497923018708371e-14, t.y + l1p));
}

// log1p(y) for finite y >= 0 (the t family's log(1 + z^2 / df)): u = 1 + y
// rounded, log1p(y) = log(u) + (y - (u - 1)) / u, the correction (below one ulp
// of u, relative to u) taken with the hardware reciprocal.
__device__ __forceinline__ double log1p_pos_tab(double y, const double2* ltab) {
  const double u = 1.0 + y;
  const double corr = (y - (u - 1.0)) * __builtin_amdgcn_rcp(u);
  return log_unit_tab(u, ltab) + corr;
}

// log(u) for u in (0, 1) (Box-Muller radius and acceptance uniforms, never 0):
// u = m 2^e with m in [1/2, 1) and e <= 0, so e ln2, log c and log1p(r) never
// cancel; c = 1/2 + j/256 the nearest table point, |r| <= 1/256, log1p to r^7.
// The LDS log table holds kBmTab's log rows, then its (0, 1) rows (load_bm_tables); at
// m ~ 1 the entry is exactly (1, 0).
__device__ __forceinline__ double log_u01_tab(double u, const double2* ltab) {
  int e;
  const double m = frexp(u, &e);
  // j = rint(256 m) - 128 in [0, 128] (= rint(256 m - 128): the shift is an even
  // integer); 256 m by ldexp, the -128 folded into the LDS read offset (an fma
  // needed its two constants in VGPRs, re-made every call)
  const double2 t = ltab[kLogN - 128 + (int)rint(ldexp(m, 8))];
  const double r = fma(m, t.x, -1.0);
  double p = 0.14285714285714285;                // 1/7
  p = hfma(p, r, -0.16666666666666666);
  p = hfma(p, r, 0.2);
  p = hfma(p, r, -0.25);
  p = hfma(p, r, 0.3333333333333333);
  p = hfma(p, r, -0.5);
  const double l1p = fma(r * r, p, r);
  const double de = (double)e;
  return fma(de, 0.6931471805598903, fma(de, 5.497923018708371e-14, t.y + l1p));
}

// sin(pi x), cos(pi x) for x in [0, 2]: x = i/128 + r, |r| <= 1/256, table
// (sin, cos)(pi i / 128) rotated by theta = pi r with short Taylor forms.
__device__ __forceinline__ void sincospi_tab(double x, double& sn, double& cs,
                                             const double2* sct) {
  const double q = rint(x * 128.0);                 // 0..256
  const double r = fma(q, -0.0078125, x);           // exact
  const double2 t = sct[(int)q];
  const double th = fma(r, 3.141592653589793, r * 1.2246467991473532e-16);
  const double t2 = th * th;
  double ps = hfma(t2, -0.0001984126984126984, 0.008333333333333333);
  ps = hfma(ps, t2, -0.16666666666666666);
  const double st = fma(th * t2, ps, th);           // sin(theta)
  double pc = hfma(t2, 2.48015873015873e-05, -0.001388888888888889);
  pc = hfma(pc, t2, 0.041666666666666664);
  pc = hfma(pc, t2, -0.5);
  const double ct = fma(t2, pc, 1.0);               // cos(theta)
  sn = fma(t.x, ct, t.y * st);
  cs = fma(t.y, ct, -(t.x * st));
}

// cos(pi x) for x = b 2^-23 (b < 2^24, so x in [0, 2)), from the integer b: table
// point q = round(b / 2^16) (= rint(128 x) up to the tie direction; either point
// keeps |r| <= 1/256) and the exact residual r = (b - q 2^16) 2^-23, as
// sincospi_tab otherwise
__device__ __forceinline__ double cospi_tab_u24(uint32_t b, const double2* sct) {
  const uint32_t q = (b + 0x8000u) >> 16;
  const double r = (double)(int)(b - (q << 16)) * 0x1p-23;
  const double2 t = sct[q];
  const double th = fma(r, 3.141592653589793, r * 1.2246467991473532e-16);
  const double t2 = th * th;
  double ps = hfma(t2, -0.0001984126984126984, 0.008333333333333333);
  ps = hfma(ps, t2, -0.16666666666666666);
  const double st = fma(th * t2, ps, th);
  double pc = hfma(t2, 2.48015873015873e-05, -0.001388888888888889);
  pc = hfma(pc, t2, 0.041666666666666664);
  pc = hfma(pc, t2, -0.5);
  const double ct = fma(t2, pc, 1.0);
  return fma(t.y, ct, -(t.x * st));
}

// Two standard normals (Box-Muller) with the table transcendentals.
__device__ __forceinline__ void normal_pair_tab(u4 w, double& z0, double& z1, const double2* sct,
                                                const double2* ltab);

// Uniforms from 52 random bits by filling the mantissa of a double in [1, 2):
//   u1 = 1.m - (1 - 2^-53) = (2m + 1) 2^-53  in (0, 1)   (never 0: log is finite)
//   u2 = 1.m - 1            = m 2^-52         in [0, 1)
__device__ __forceinline__ double unit_mantissa(uint32_t lo, uint32_t hi) {
  const uint32_t mlo = __builtin_amdgcn_alignbit(hi, lo, 12);
  const uint32_t mhi = (hi >> 12) | 0x3FF00000u;
  return __hiloint2double((int)mhi, (int)mlo);
}

__device__ __forceinline__ void normal_pair_tab(u4 w, double& z0, double& z1, const double2* sct,
                                                const double2* ltab) {
  const double u1 = unit_mantissa(w.x, w.y) - 0x1.fffffffffffffp-1;
  const double u2 = unit_mantissa(w.z, w.w) - 1.0;
  const double r = sqrt_pos(-2.0 * log_u01_tab(u1, ltab));
  double s, c;
  sincospi_tab(2.0 * u2, s, c, sct);
  z0 = r * c;
  z1 = r * s;
}

// Fill the LDS tables (all threads of the block; caller synchronises): rows
// [0, kSinCosN) of kBmTab to sct, the rest to ltab.
__device__ __forceinline__ void load_bm_tables(double2* sct, double2* ltab) {
  auto dst = [&](int i) { return i < kSinCosN ? sct + i : ltab + (i - kSinCosN); };
  const double2* src = reinterpret_cast<const double2*>(kBmTab);
  const int t = threadIdx.x, nt = blockDim.x;
  if (2 * nt >= kBmTabN) {
    // both of a thread's rows loaded before either is stored: one memory latency
    // for the whole fill (a loop per table waited for every load in turn)
    const int i0 = t, i1 = t + nt;
    const double2 v0 = src[i0 < kBmTabN ? i0 : 0];
    const double2 v1 = src[i1 < kBmTabN ? i1 : 0];
    if (i0 < kBmTabN) *dst(i0) = v0;
    if (i1 < kBmTabN) *dst(i1) = v1;
  } else {
    for (int i = t; i < kBmTabN; i += nt) *dst(i) = src[i];
  }
}

// Two standard normals from one Philox block (Box-Muller).
__device__ __forceinline__ void normal_pair(u4 w, double& z0, double& z1) {
  const double u1 = unit_mantissa(w.x, w.y) - 0x1.fffffffffffffp-1;
  const double u2 = unit_mantissa(w.z, w.w) - 1.0;
  const double r = sqrt_pos(-2.0 * log_unit(u1));
  double s, c;
  sincospi_unit(2.0 * u2, s, c);
  z0 = r * c;
  z1 = r * s;
}

// Gamma(shape) draws for the two elements of a column pair (Marsaglia-Tsang,
// ACM TOMS 26(3) 2000).  Proposal k uses Philox purpose 1+k; each proposal
// block gives two 32-bit-uniform Box-Muller normals and two uniforms.
// TAB: use the LDS-table log / sincos (sct, ltab) instead of the short forms
// and the general log of the acceptance test.
template <bool TAB = false>
__device__ __forceinline__ void gamma_pair(const Rng& rng, uint32_t pair, uint32_t sample,
                                           uint32_t step, double shape, double& ga,
                                           double& gb, const double2* sct = nullptr,
                                           const double2* ltab = nullptr) {
  const double d = shape - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  bool da = false, db = false;
  ga = d;
  gb = d;
  for (uint32_t k = 0; k < 64u && !(da && db); ++k) {
    const u4 w = rng.draw(pair, sample, step, 1u + k);
    const double u1 = ((double)w.x + 0.5) * 0x1p-32;
    const double u2 = (double)w.y * 0x1p-32;
    double s, cs, r;
    if constexpr (TAB) {
      r = sqrt_pos(-2.0 * log_u01_tab(u1, ltab));
      sincospi_tab(2.0 * u2, s, cs, sct);
    } else {
      r = sqrt_pos(-2.0 * log_unit(u1));
      sincospi_unit(2.0 * u2, s, cs);
    }
    const double za = r * cs, zb = r * s;
    const double ua = ((double)w.z + 0.5) * 0x1p-32;
    const double ub = ((double)w.w + 0.5) * 0x1p-32;
    if (!da) {
      double v = 1.0 + c * za;
      if (v > 0.0) {
        v = v * v * v;
        const double lu = TAB ? log_u01_tab(ua, ltab) : log(ua);
        const double lv = (TAB && v >= 0x1p-1022 && v < 0x1p+1023) ? log_unit_tab(v, ltab) : log(v);
        if (lu < 0.5 * za * za + d - d * v + d * lv) {
          ga = d * v;
          da = true;
        }
      }
    }
    if (!db) {
      double v = 1.0 + c * zb;
      if (v > 0.0) {
        v = v * v * v;
        const double lu = TAB ? log_u01_tab(ub, ltab) : log(ub);
        const double lv = (TAB && v >= 0x1p-1022 && v < 0x1p+1023) ? log_unit_tab(v, ltab) : log(v);
        if (lu < 0.5 * zb * zb + d - d * v + d * lv) {
          gb = d * v;
          db = true;
        }
      }
    }
  }
}

// ---- Bailey t draws (the t family's log-weight draws) -----------------------
// Bailey, "Polar generation of random variates with the t-distribution", Math.
// Comp. 62 (1994) 779-781: for U1, U2 iid U(0, 1),
//   T = cos(2 pi U2) sqrt(df (U1^(-2/df) - 1))  ~  t(df)
// (the polar method's radius W = U1 and angle drawn directly: no rejection, no
// divergent loop).  One Philox block per column pair j of row n, counter (j, n,
// step, stream | kBaileyPurpose << 24): variate 2 j from words (x, z), 2 j + 1
// from (y, w); of each (lo, hi) pair U1 = (a + 1/2) 2^-40 with a = lo | (hi & 0xff)
// << 32, and U2 = (hi >> 8) 2^-24 (|T| reaches sqrt(df (2^(82/df) - 1)): 11.2 at
// df = 40, past the t(40) quantile of 1 - 1e-13).  Per variate one log, one exp,
// one sin / cos pair, a square root and log q's log1p(T^2 / df) = log1p(cos^2
// (U1^(-2/df) - 1)) -- a Box-Muller normal and Marsaglia-Tsang gamma attempts (each
// a normal and two logs) before.  oracle/vbrng.c (family 2) restates it with libm.
constexpr uint32_t kBaileyPurpose = 65u;

// T of words (lo, hi) and l1 = log1p(T^2 / df); c2 = -2 / df (formed on the host
// as the oracle forms it)
__device__ __forceinline__ double bailey_t(uint32_t lo, uint32_t hi, double df, double c2,
                                           const double2* sct, const double2* ltab, double& l1) {
  const double a = hfma((double)(hi & 0xffu), 0x1p32, (double)lo);  // exact, 40 bits
  const double u1 = hfma(a, 0x1p-40, 0x1p-41);                        // (a + 1/2) 2^-40
  const double em1 = expm1_pos(c2 * log_u01_tab(u1, ltab));           // U1^(-2/df) - 1
  const double cs = cospi_tab_u24(hi >> 8, sct);                      // cos(2 pi U2)
  l1 = log1p_pos_tab(cs * cs * em1, ltab);
  return cs * sqrt_pos(df * em1);
}

// T of words (lo, hi) and y = T^2 / df (the log-q argument: log1p(y)), for callers that
// multiply the (1 + y) of a row's variates and take one log of the product
__device__ __forceinline__ double bailey_t_y(uint32_t lo, uint32_t hi, double df, double c2,
                                             const double2* sct, const double2* ltab, double& y) {
  const double a = hfma((double)(hi & 0xffu), 0x1p32, (double)lo);  // exact, 40 bits
  const double u1 = hfma(a, 0x1p-40, 0x1p-41);                        // (a + 1/2) 2^-40
  const double em1 = expm1_pos(c2 * log_u01_tab(u1, ltab));           // U1^(-2/df) - 1
  const double cs = cospi_tab_u24(hi >> 8, sct);                      // cos(2 pi U2)
  y = cs * cs * em1;
  return cs * sqrt_pos(df * em1);
}

// ---- wave-level helpers (wave64) -------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Wave-wide sum of a double with DPP row ops + gfx950 permlane swaps (no LDS
// traffic, short latency).  Every lane ends with the bitwise-identical total.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double swap_sum16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}

__device__ __forceinline__ double swap_sum32(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}

__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  v = swap_sum16(v);       // rows 0+1, 2+3
  return swap_sum32(v);    // halves
}

// Sum over lanes l = c (mod 4) of a group of 64/PPW lanes (all lanes of the
// group receive their residue class's total).
template <int PPW>
__device__ __forceinline__ double stride4_sum(double k) {
  k += dpp_f64<0x124>(k);  // row_ror:4
  k += dpp_f64<0x128>(k);  // row_ror:8
  if constexpr (PPW <= 2) k = swap_sum16(k);  // rows 0+1, 2+3
  if constexpr (PPW == 1) k = swap_sum32(k);  // halves
  return k;
}

// max(a, b) as one v_max_f64: fmax's lowering first canonicalises each operand
// (v_max_f64 x, x, x -- signalling-NaN quieting) and arithmetic never yields a
// signalling NaN, so the canonicalisations only lengthen the wave reductions'
// chains; quiet NaNs behave as in fmax (the other operand is returned)
__device__ __forceinline__ double fmax_raw(double a, double b) {
  double d;
  asm("v_max_f64 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

__device__ __forceinline__ double swap_max16(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return fmax_raw(__hiloint2double((int)b[0], (int)a[0]), __hiloint2double((int)b[1], (int)a[1]));
}

__device__ __forceinline__ double swap_max32(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return fmax_raw(__hiloint2double((int)b[0], (int)a[0]), __hiloint2double((int)b[1], (int)a[1]));
}

// Wave-wide max with DPP + permlane swaps (every lane receives the maximum).
__device__ __forceinline__ double wave_max_dpp(double v) {
  v = fmax_raw(v, dpp_f64<0xB1>(v));
  v = fmax_raw(v, dpp_f64<0x4E>(v));
  v = fmax_raw(v, dpp_f64<0x141>(v));
  v = fmax_raw(v, dpp_f64<0x140>(v));
  v = swap_max16(v);
  return swap_max32(v);
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// numpy's logaddexp (npy_logaddexp): equal args -> x + log 2.
__device__ __forceinline__ double logaddexp(double x, double y) {
  if (x == y) return x + kLn2;
  const double t = x - y;
  if (t > 0) return x + log1p(exp(-t));
  if (t <= 0) return y + log1p(exp(t));
  return t;  // NaN
}

// ---- targets -----------------------------------------------------------------
// Separable targets expose a per-coordinate log density + derivative (lp1);
// every target exposes a row evaluation (row) for D <= kRowMax.

struct IsoGauss {  // N(0, I): log p = sum_d -x_d^2/2 - log(2 pi)/2
  static constexpr bool kSeparable = true;
  __device__ __forceinline__ static double lp1(double x, double& g) {
    g = -x;
    return -0.5 * x * x - 0.5 * kLog2Pi;
  }
};

// normal-mixture.ipynb cell 2: logaddexp(N(x;-2,1), N(x;2,1)) - log 2, per coordinate.
struct Mixture {
  static constexpr bool kSeparable = true;
  __device__ __forceinline__ static double lp1(double x, double& g) {
    const double a = -0.5 * (x + 2.0) * (x + 2.0) - 0.5 * kLog2Pi;
    const double b = -0.5 * (x - 2.0) * (x - 2.0) - 0.5 * kLog2Pi;
    // one exp serves both terms: with t = a - b (= -4x) and e = exp(-|t|),
    // logaddexp(a, b) = max(a, b) + log1p(e) (numpy's form; t = 0 gives
    // log1p(1) = log 2) and the posterior weight of the +2 component
    // 1 / (1 + exp(t)) = 1 / (1 + e) for t <= 0, e / (1 + e) for t > 0
    const double t = a - b;
    const double e = exp_fast(-fabs(t));
    // e in (0, 1]: a refined reciprocal and the table-free log1p (~1 ulp each)
    // instead of an IEEE division and the library's double-double log1p, which were
    // most of a row's dependent chain in the block kernel (config 1)
    const double d = 1.0 + e;
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    r = fma(r, fma(-d, r, 1.0), r);
    const double wb = t > 0.0 ? e * r : r;
    g = -(x + 2.0) + 4.0 * wb;
    return (t > 0.0 ? a : b) + log1p_pos_fast(e) - kLn2;
  }
};

// funnel-distribution.ipynb cell 2, generalised to D: x[1] = log sigma ~ N(0, 1.35^2),
// every other coordinate ~ N(0, exp(log sigma)^2).
struct Funnel {
  static constexpr bool kSeparable = false;
  template <int DMAX>
  __device__ __forceinline__ static double row(const double* x, double* g, int D) {
    constexpr double s0 = 1.35;
    const double v = x[1];
    const double zv = v / s0;
    double lp = -0.5 * zv * zv - log(s0) - 0.5 * kLog2Pi;
    double gv = -zv / s0;
    const double inv_s = exp_fast(-v);
    const double inv_s2 = inv_s * inv_s;
    // branch-free over the DMAX slots (the D < DMAX tail is masked by selects)
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d == 1) continue;
      const double z = x[d] * inv_s;
      const bool on = d < D;
      lp += on ? -0.5 * z * z - v - 0.5 * kLog2Pi : 0.0;
      g[d] = on ? -x[d] * inv_s2 : 0.0;
      gv += on ? z * z - 1.0 : 0.0;
    }
    g[1] = gv;
    return lp;
  }
  // Split rows (block_kernel, lanes 2j / 2j + 1 of a pair): this lane's log p part
  // and the gradients of its coordinates [h DH, h DH + DH) (xh / gh); x1 = log sigma
  // is computed by both lanes.  The pair's gv parts are summed with one DPP swap
  // (both lanes active) and land on coordinate 1's owner.
  template <int DH>
  __device__ __forceinline__ static void lane_const(int /*h*/, double* /*lk*/) {}
  template <int DMAX, int DH>
  __device__ __forceinline__ static double row_half(const double* xh, double* gh, int h, int D,
                                                    double /*x0*/, double x1,
                                                    const double* /*lk*/) {
    constexpr double s0 = 1.35, is0 = 1.0 / 1.35;
    const double v = x1;
    // (multiplications by 1 / 1.35 rounded at compile time instead of two IEEE
    // divisions on the rows' chain: within an ulp)
    const double zv = v * is0;
    double lp = h == 0 ? -0.5 * zv * zv - log(s0) - 0.5 * kLog2Pi : 0.0;
    double gv = h == 0 ? -zv * is0 : 0.0;
    const double inv_s = exp_fast(-v);
    const double inv_s2 = inv_s * inv_s;
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      const int d = h * DH + k;
      const bool on = d < D && d != 1;
      const double z = xh[k] * inv_s;
      lp += on ? -0.5 * z * z - v - 0.5 * kLog2Pi : 0.0;
      gh[k] = on ? -xh[k] * inv_s2 : 0.0;
      gv += on ? z * z - 1.0 : 0.0;
    }
    gv += dpp_f64<0xB1>(gv);   // quad_perm [1,0,3,2]: the pair's other lane
    constexpr int h1 = DH >= 2 ? 0 : 1, k1 = DH >= 2 ? 1 : 0;
    if (h == h1) gh[k1] = gv;
    return lp;
  }
};

// eight_schools_ncp.stan:1-23 log_prob (constants of the ~ statements dropped,
// log-Jacobian of tau = exp(u) added), unconstrained order [mu, log tau, theta_tilde(8)].
struct EightSchools {
  static constexpr bool kSeparable = false;
  template <int DMAX>
  __device__ __forceinline__ static double row(const double* x, double* g, int /*D*/) {
    const double y[8] = {28., 8., -3., 7., -1., 1., 18., 12.};
    // 1 / sigma_j rounded at compile time: multiplications instead of 24 fp64
    // divisions per row (within an ulp of the divided forms)
    constexpr double is[8] = {1. / 15., 1. / 10., 1. / 16., 1. / 11.,
                              1. / 9.,  1. / 11., 1. / 10., 1. / 18.};
    const double mu = x[0], u = x[1], tau = exp_fast(u);
    const double t5 = tau * 0.2, m5 = mu * 0.2;
    double lp = -0.5 * m5 * m5 - log1p(t5 * t5) + u;
    double gmu = -m5 * 0.2;
    double gu = -2.0 * t5 * t5 / (1.0 + t5 * t5) + 1.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double th = x[2 + j];
      const double r = (y[j] - mu - tau * th) * is[j];
      const double rs = r * is[j];  // r / sigma_j
      lp += -0.5 * th * th - 0.5 * r * r;
      gmu += rs;
      gu += rs * (tau * th);
      g[2 + j] = -th + rs * tau;
    }
    g[0] = gmu;
    g[1] = gu;
    return lp;
  }
  // log p alone with the LDS log table (log-weight kernels, which load the
  // Box-Muller tables and discard the gradient): log1p(t5^2) through
  // log1p_pos_tab (~1 ulp) instead of the double-double library log1p, which was
  // ~100 of a draw row's ~2 500 instructions; non-finite arguments take the
  // library form
  template <int DMAX>
  __device__ __forceinline__ static double lp_tab(const double* x, int /*D*/, const double2* lt) {
    constexpr double y[8] = {28., 8., -3., 7., -1., 1., 18., 12.};
    constexpr double is[8] = {1. / 15., 1. / 10., 1. / 16., 1. / 11.,
                              1. / 9.,  1. / 11., 1. / 10., 1. / 18.};
    const double mu = x[0], u = x[1], tau = exp_fast(u);
    const double t5 = tau * 0.2, m5 = mu * 0.2;
    const double w = t5 * t5;
    double l1;
    if (w < 0x1p+1000) l1 = log1p_pos_tab(w, lt);
    else l1 = log1p(w);
    double lp = -0.5 * m5 * m5 - l1 + u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double th = x[2 + j];
      const double r = (y[j] - mu - tau * th) * is[j];
      lp += -0.5 * th * th - 0.5 * r * r;
    }
    return lp;
  }
  // Split rows (see Funnel::row_half): lane 0 owns mu, log tau and theta_tilde
  // 0-2, lane 1 theta_tilde 3-7 (DH = 5); both compute tau.  The pair's mu and
  // log tau gradient parts are summed with one DPP swap each.
  // lk: the lane's y_j and 1 / sigma_j (lane_const), made once per thread before
  // the step loop.  Selected here per row (h ? y[j1] : y[j0]), the compiler turned
  // them into loads from a constant table at a per-lane index: ten global loads,
  // reissued after every row's LDS reads and waited for on the row's chain.
  template <int DH>
  __device__ __forceinline__ static void lane_const(int h, double* lk) {
    static_assert(DH >= 2, "eight schools: coordinates 0 and 1 on lane 0");
    constexpr double y[8] = {28., 8., -3., 7., -1., 1., 18., 12.};
    constexpr double is[8] = {1. / 15., 1. / 10., 1. / 16., 1. / 11.,
                              1. / 9.,  1. / 11., 1. / 10., 1. / 18.};
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      // theta_tilde j = h DH + k - 2: lane 0's k >= 2, every k of lane 1
      const int j0 = k >= 2 ? k - 2 : 0, j1 = DH + k - 2 < 8 ? DH + k - 2 : 7;
      double yj = h ? y[j1] : y[j0], isj = h ? is[j1] : is[j0];
      asm("" : "+v"(yj), "+v"(isj));   // (opaque: kept in registers, not re-derived per row)
      lk[k] = yj;
      lk[DH + k] = isj;
    }
  }
  template <int DMAX, int DH>
  __device__ __forceinline__ static double row_half(const double* xh, double* gh, int h, int /*D*/,
                                                    double x0, double x1, const double* lk) {
    const double mu = x0, u = x1, tau = exp_fast(u);
    const double t5 = tau * 0.2, m5 = mu * 0.2;
    // prior terms of mu and tau on lane 0, computed by both lanes without a branch
    // (lane 1's discarded by the selects): as a lane-0 block they could not be
    // interleaved with the theta terms below, which depend only on tau as well
    // (the table-free log1p and a refined reciprocal instead of the library log1p
    // and an IEEE division, ~1 ulp; also branch-free at the extremes: for w >= 2^1000
    // the rounding correction of 1 + w is 0 and log_unit takes any normal argument,
    // w = inf gives inf by the select and NaN stays NaN; the gradient
    // -2 w / (1 + w) + 1 is NaN at w = inf, as the divided form is)
    const double w = t5 * t5;
    const double dw = 1.0 + w;
    double rw = __builtin_amdgcn_rcp(dw);
    rw = fma(rw, fma(-dw, rw, 1.0), rw);
    rw = fma(rw, fma(-dw, rw, 1.0), rw);
    const double l1 = w < INFINITY ? log1p_pos_fast(w) : w;
    const double gu0 = -2.0 * w * rw + 1.0;
    double lp = h == 0 ? -0.5 * m5 * m5 - l1 + u : 0.0;
    double gmu = h == 0 ? -m5 * 0.2 : 0.0;
    double gu = h == 0 ? gu0 : 0.0;
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      const bool th_on = h == 1 || k >= 2;
      const double yj = lk[k], isj = lk[DH + k];
      const double th = xh[k];
      const double r = (yj - mu - tau * th) * isj;
      const double rs = r * isj;
      lp += th_on ? -0.5 * th * th - 0.5 * r * r : 0.0;
      gmu += th_on ? rs : 0.0;
      gu += th_on ? rs * (tau * th) : 0.0;
      gh[k] = th_on ? -th + rs * tau : 0.0;
    }
    gmu += dpp_f64<0xB1>(gmu);
    gu += dpp_f64<0xB1>(gu);
    if (h == 0) {
      gh[0] = gmu;
      gh[1] = gu;
    }
    return lp;
  }
};

// Row evaluation for separable targets.
template <class T>
struct SepRow {
  template <int DMAX>
  __device__ __forceinline__ static double row(const double* x, double* g, int D) {
    double lp = 0.0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      double gd;
      const double l = T::lp1(x[d], gd);
      const bool on = d < D;
      lp += on ? l : 0.0;
      g[d] = on ? gd : 0.0;
    }
    return lp;
  }
  // Split rows: this lane's coordinates [h DH, h DH + DH) only (no cross terms)
  template <int DH>
  __device__ __forceinline__ static void lane_const(int /*h*/, double* /*lk*/) {}
  template <int DMAX, int DH>
  __device__ __forceinline__ static double row_half(const double* xh, double* gh, int h, int D,
                                                    double /*x0*/, double /*x1*/,
                                                    const double* /*lk*/) {
    double lp = 0.0;
#pragma unroll
    for (int k = 0; k < DH; ++k) {
      double gd;
      const double l = T::lp1(xh[k], gd);
      const bool on = h * DH + k < D;
      lp += on ? l : 0.0;
      gh[k] = on ? gd : 0.0;
    }
    return lp;
  }
};

// Windowed adagrad update of coordinate p (vb.py:365-374, the reference's
// "adagrad" step): store g in the ring slot of this step, q = sum over the last
// min(step + 1, W) slots of (scale_k g_k)^2, oldest first, and return
// lam - lr g / sqrt(eps + q).  Shared by adagrad_update_kernel and the fused
// gradient + update pass of the materialised mean-field path.
__device__ __forceinline__ double adagrad_step(long long p, long long P, double lam, double g,
                                               double* ring, int W, long long step, double lr,
                                               double eps, const double* scale) {
  const int slot = (int)(step % W);
  ring[(long long)slot * P + p] = g;
  const int cnt = (step + 1 < W) ? (int)(step + 1) : W;
  const int oldest = (cnt < W) ? 0 : (int)((step + 1) % W);
  double q = 0.0;
  for (int k = 0; k < cnt; ++k) {
    int L = oldest + k;
    if (L >= W) L -= W;
    double t = L == slot ? g : ring[(long long)L * P + p];
    if (scale) t = __dmul_rn(scale[k], t);
    q = __dadd_rn(q, __dmul_rn(t, t));
  }
  return __dsub_rn(lam, __dmul_rn(lr, g) / sqrt(__dadd_rn(eps, q)));
}

}  // namespace vbd

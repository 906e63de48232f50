/*
 * vbrng.c -- ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the product.
 *
 * Plain-C restatement of the counter-based noise the HIP kernels draw in
 * VB_NOISE_PHILOX mode, so tests can regenerate the exact draws on the CPU
 * and compare kernel results against the numpy restatement of the reference
 * algorithm (oracle/vb_oracle.py) on identical noise.
 *
 *  - Philox4x32-10: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as
 *    easy as 1, 2, 3", SC'11 (Random123).  Pinned by the Random123 known-answer
 *    vectors in tests/test_oracle_rng.py.
 *  - counter = (pair j, sample n, step, stream | purpose << 24), key = seed.
 *  - normal pair: Box-Muller on 52-bit mantissa-fill uniforms u1 = (2m+1)2^-53,
 *    u2 = m 2^-52 (m the top 52 bits of a 64-bit half of the block).
 *  - t draw: sqrt(df/2) * gauss / sqrt(gamma(df/2)), the structure of numpy's
 *    legacy standard_t; gamma by Marsaglia & Tsang (2000), proposals from
 *    purposes 1..64 with 32-bit uniforms.
 *  - Bailey t draw (family 2; the log-weight draws of the t family): Bailey,
 *    "Polar generation of random variates with the t-distribution", Math. Comp.
 *    62 (1994) 779-781: T = cos(2 pi U2) sqrt(df (U1^(-2/df) - 1)) for U1, U2 iid
 *    U(0, 1).  Column pair j of row n from the block at counter (j, n, step,
 *    stream | 65 << 24): variate 2j from words (x, z), 2j + 1 from (y, w); of each
 *    (lo, hi), U1 = (a + 1/2) 2^-40 with a = lo | (hi & 0xff) << 32 and
 *    U2 = (hi >> 8) 2^-24; T = cos(2 pi U2) sqrt(df expm1(-(2/df) log U1)).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { uint32_t v[4]; } blk;

static blk philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t a = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t b = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t y0 = (uint32_t)(b >> 32) ^ c1 ^ k0;
    uint32_t y1 = (uint32_t)b;
    uint32_t y2 = (uint32_t)(a >> 32) ^ c3 ^ k1;
    uint32_t y3 = (uint32_t)a;
    c0 = y0; c1 = y1; c2 = y2; c3 = y3;
  }
  blk o = {{c0, c1, c2, c3}};
  return o;
}

void vbo_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  blk b = philox(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
  for (int i = 0; i < 4; ++i) out[i] = b.v[i];
}

static blk draw(uint64_t seed, uint32_t stream, uint32_t pair, uint32_t n, uint32_t step,
                uint32_t purpose) {
  return philox(pair, n, step, (stream & 0x00FFFFFFu) | (purpose << 24), (uint32_t)seed,
                (uint32_t)(seed >> 32));
}

/* 52 random bits into the mantissa of a double in [1, 2) */
static double unit_mantissa(uint32_t lo, uint32_t hi) {
  uint64_t bits = 0x3FF0000000000000ull | (((((uint64_t)hi) << 32) | lo) >> 12);
  double d;
  memcpy(&d, &bits, sizeof d);
  return d;
}

static void gauss2(blk w, double* z0, double* z1) {
  double u1 = unit_mantissa(w.v[0], w.v[1]) - 0x1.fffffffffffffp-1; /* (2m+1) 2^-53 */
  double u2 = unit_mantissa(w.v[2], w.v[3]) - 1.0;                  /* m 2^-52 */
  double r = sqrt(-2.0 * log(u1));
  double th = 2.0 * M_PI * u2;
  *z0 = r * cos(th);
  *z1 = r * sin(th);
}

static void gamma2(uint64_t seed, uint32_t stream, uint32_t pair, uint32_t n, uint32_t step,
                   double shape, double* ga, double* gb) {
  double d = shape - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  int okA = 0, okB = 0;
  *ga = d;
  *gb = d;
  for (uint32_t k = 0; k < 64u && !(okA && okB); ++k) {
    blk w = draw(seed, stream, pair, n, step, 1u + k);
    double u1 = ((double)w.v[0] + 0.5) * 0x1p-32;
    double u2 = (double)w.v[1] * 0x1p-32;
    double r = sqrt(-2.0 * log(u1)), th = 2.0 * M_PI * u2;
    double z[2] = {r * cos(th), r * sin(th)};
    double u[2] = {((double)w.v[2] + 0.5) * 0x1p-32, ((double)w.v[3] + 0.5) * 0x1p-32};
    int* ok[2] = {&okA, &okB};
    double* g[2] = {ga, gb};
    for (int e = 0; e < 2; ++e) {
      if (*ok[e]) continue;
      double v = 1.0 + c * z[e];
      if (v <= 0.0) continue;
      v = v * v * v;
      if (log(u[e]) < 0.5 * z[e] * z[e] + d - d * v + d * log(v)) {
        *g[e] = d * v;
        *ok[e] = 1;
      }
    }
  }
}

#define VBO_BAILEY_PURPOSE 65u

/* Bailey t variates of column pair j of row n (see the header) */
static void bailey_pair(uint64_t seed, uint32_t stream, uint32_t j, uint32_t n, uint32_t step,
                        double df, double* t0, double* t1) {
  blk w = draw(seed, stream, j, n, step, VBO_BAILEY_PURPOSE);
  double* out[2] = {t0, t1};
  for (int c = 0; c < 2; ++c) {
    uint32_t lo = w.v[c], hi = w.v[2 + c];
    double a = (double)((((uint64_t)(hi & 0xffu)) << 32) | lo);
    double u1 = (a + 0.5) * 0x1p-40;
    double u2 = (double)(hi >> 8) * 0x1p-24;
    *out[c] = cos(2.0 * M_PI * u2) * sqrt(df * expm1((-2.0 / df) * log(u1)));
  }
}

/* standardized draws eps[n][D] for one step: family 0 = N(0,1), 1 = t(df),
 * 2 = Bailey t(df) (the log-weight draws) */
void vbo_fill(uint64_t seed, uint32_t stream, uint32_t step, int64_t nrows, int64_t D, int family,
              double df, double* eps) {
  int64_t npairs = (D + 1) / 2;
  if (family == 2) {
    for (int64_t r = 0; r < nrows; ++r)
      for (int64_t j = 0; j < npairs; ++j) {
        double t0, t1;
        bailey_pair(seed, stream, (uint32_t)j, (uint32_t)r, step, df, &t0, &t1);
        eps[r * D + 2 * j] = t0;
        if (2 * j + 1 < D) eps[r * D + 2 * j + 1] = t1;
      }
    return;
  }
  for (int64_t r = 0; r < nrows; ++r) {
    for (int64_t j = 0; j < npairs; ++j) {
      double z0, z1;
      gauss2(draw(seed, stream, (uint32_t)j, (uint32_t)r, step, 0u), &z0, &z1);
      if (family == 1) {
        double ga, gb;
        gamma2(seed, stream, (uint32_t)j, (uint32_t)r, step, df / 2.0, &ga, &gb);
        double s = sqrt(df / 2.0);
        z0 = s * z0 / sqrt(ga);
        z1 = s * z1 / sqrt(gb);
      }
      eps[r * D + 2 * j] = z0;
      if (2 * j + 1 < D) eps[r * D + 2 * j + 1] = z1;
    }
  }
}

/* full-rank t scale draws s[n] = sqrt(chisquare(df)/df) = sqrt(2 Gamma(df/2)/df)
 * from the reserved column pair 0xFFFFFFFF (vb_fr.hip fr_noise_kernel) */
void vbo_fr_scale(uint64_t seed, uint32_t stream, uint32_t step, int64_t nrows, double df,
                  double* s) {
  for (int64_t r = 0; r < nrows; ++r) {
    double ga, gb;
    gamma2(seed, stream, 0xFFFFFFFFu, (uint32_t)r, step, df / 2.0, &ga, &gb);
    s[r] = sqrt(2.0 * ga / df);
  }
}

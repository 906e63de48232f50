/*
 * sanitize_main.c -- ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Driver for an AddressSanitizer + UndefinedBehaviorSanitizer build of the C
 * noise oracle (vbrng.c, compiled into this translation unit): the Random123
 * known-answer vectors, then every entry point over ragged shapes (odd D, so the
 * last column pair has no second element; zero rows; one row; the t family with
 * its gamma rejection loop; the full-rank scale draws).  Each draw array is
 * allocated with its exact size, so a write past its end is an ASan report.  The
 * draws are printed as hex bit patterns for tests/test_oracle_sanitize.py, which
 * compares them with the plain build (liboracle_rng.so).
 *
 *   gcc -std=gnu11 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all \
 *       -fno-omit-frame-pointer -ffp-contract=off -o vbrng_asan sanitize_main.c -lm
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vbrng.c"

static int kat(void) {
  static const uint32_t ctr[3][4] = {{0, 0, 0, 0},
                                     {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu},
                                     {0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u}};
  static const uint32_t key[3][2] = {{0, 0}, {0xffffffffu, 0xffffffffu}, {0xa4093822u, 0x299f31d0u}};
  static const uint32_t want[3][4] = {{0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u},
                                      {0x408f276du, 0x41c83b0eu, 0xa20bc7c6u, 0x6d5451fdu},
                                      {0xd16cfe09u, 0x94fdccebu, 0x5001e420u, 0x24126ea1u}};
  for (int i = 0; i < 3; ++i) {
    uint32_t out[4];
    vbo_philox(ctr[i], key[i], out);
    if (memcmp(out, want[i], sizeof out) != 0) {
      fprintf(stderr, "KAT %d mismatch\n", i);
      return 1;
    }
  }
  return 0;
}

static void dump(const char* tag, const double* v, int64_t n) {
  printf("%s %lld", tag, (long long)n);
  for (int64_t i = 0; i < n; ++i) {
    uint64_t b;
    memcpy(&b, v + i, sizeof b);
    printf(" %016llx", (unsigned long long)b);
  }
  printf("\n");
}

int main(void) {
  if (kat()) return 1;
  printf("kat ok\n");
  /* (seed, stream, step, rows, D, family, df) */
  const struct { uint64_t seed; uint32_t stream, step; int64_t rows, D; int fam; double df; } cases[] = {
      {0, 1, 0, 3, 1, 0, 0.0},       {7, 5, 11, 5, 7, 0, 0.0},  {123456789ull, 3, 2, 4, 9, 1, 40.0},
      {1ull << 40, 2, 1, 2, 3, 1, 3.0}, {42, 9, 0, 0, 5, 0, 0.0}, {42, 9, 4, 1, 16, 1, 100.0},
  };
  for (size_t c = 0; c < sizeof cases / sizeof cases[0]; ++c) {
    const int64_t n = cases[c].rows * cases[c].D;
    double* eps = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    vbo_fill(cases[c].seed, cases[c].stream, cases[c].step, cases[c].rows, cases[c].D, cases[c].fam,
             cases[c].df, eps);
    char tag[32];
    snprintf(tag, sizeof tag, "fill%zu", c);
    dump(tag, eps, n);
    free(eps);
  }
  {
    const int64_t rows = 6;
    double* s = (double*)malloc(sizeof(double) * rows);
    vbo_fr_scale(99, 4, 3, rows, 100.0, s);
    dump("frscale", s, rows);
    free(s);
  }
  return 0;
}

/* Kernel-lab check (not product code): the three-instruction division by a small constant D used by
 * compress_fused.hip (q0 = x * RN(1/D); r = fma(-q0, D, x); q = fma(r, RN(1/D), q0)) against the IEEE
 * quotient x / D, exhaustively over all 2^32 fp32 bit patterns, D = 2..15.  Result (gcc -O2
 * -ffp-contract=off -fopenmp, 8 threads, ~5 min): equal except x = +-inf (3 per D incl. -0) and, for
 * D = 6, 10, 12, 14, |x| < 2^-124 -- the ranges the kernel routes to the IEEE division.
 * Build: gcc -O2 -march=native -ffp-contract=off -fopenmp tools/check_div_const.c -o /tmp/div -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(void) {
  long long bad_total = 0;
  for (int d = 2; d <= 15; ++d) {
    const float fd = (float)d, y = 1.0f / fd;
    long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (int64_t i = 0; i < (1LL << 32); ++i) {
      uint32_t u = (uint32_t)i;
      float x;
      memcpy(&x, &u, 4);
      if (isnan(x)) continue;
      float q = x / fd;
      float q0 = x * y;
      float r = fmaf(-q0, fd, x);
      float q1 = fmaf(r, y, q0);
      uint32_t a, b;
      memcpy(&a, &q, 4);
      memcpy(&b, &q1, 4);
      if (a != b) ++bad;
    }
    printf("d=%d mismatches=%lld\n", d, bad);
    fflush(stdout);
    bad_total += bad;
  }
  printf("total %lld\n", bad_total);
  return 0;
}

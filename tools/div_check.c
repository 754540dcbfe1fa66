/* div_check.c — div_rn (kernels.hip) against IEEE division on the host: q0 = RN(w r) with
 * r = RN(1/d), two FMA residual corrections, compared bit for bit with w / d on random operands
 * over 2^-60 .. 2^60 and on near-midpoint quotients (w = q d and its neighbours) for the
 * diagonals of the SPEC grids (6, 4 + 2 eps, ...). Dev tool, not part of libpamg.
 *   gcc -O2 -ffp-contract=off -o /tmp/div_check tools/div_check.c -lm && /tmp/div_check */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rexp(int span) {
    uint64_t u = rnd();
    double d;
    u = (u & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - span + (rnd() % (2 * span))) << 52);
    memcpy(&d, &u, 8);
    return d;
}
static double div_rn(double w, double d, double r) {
    const double q0 = w * r, e0 = fma(-q0, d, w), q1 = fma(e0, r, q0), e1 = fma(-q1, d, w);
    return fma(e1, r, q1);
}
int main(void) {
    const double ds[8] = {6.0, 4.002, 3.0, 7.0, 0.1, 1.0 / 3.0, 6.000000000000001, 5.999999999999999};
    long bad = 0, n = 0;
    for (long i = 0; i < 200000000; ++i, ++n) {  /* random operands */
        const double d = (i % 3 == 0) ? ds[i % 8] : fabs(rexp(60)), w = rexp(60);
        bad += div_rn(w, d, 1.0 / d) != w / d;
    }
    for (long i = 0; i < 100000000; ++i, ++n) {  /* quotients at / next to representable values */
        const double d = ds[i % 8];
        double w = rexp(30) * d;
        const int k = (int)(rnd() % 5) - 2;
        for (int j = 0; j < abs(k); ++j) w = nextafter(w, k > 0 ? INFINITY : -INFINITY);
        bad += div_rn(w, d, 1.0 / d) != w / d;
    }
    printf("{\"cases\": %ld, \"mismatches\": %ld}\n", n, bad);
    return bad != 0;
}

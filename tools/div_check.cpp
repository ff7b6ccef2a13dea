// div_check.cpp — host check of the candidate loop's division scheme (csrc/pp_math.h div_rcp*):
// with r = RN(1/d) the Markstein quotient q = fma(fma(-q0, d, n), r, q0), q0 = n r, equals the
// IEEE quotient n / d; and one Markstein reciprocal step r1 = fma(fma(-d, r0, 1), r0, r0) turns
// an r0 within 2 ulp of 1/d into RN(1/d). Random mantissas over the exponent range the loop uses.
// Build: g++ -O2 -mfma -ffp-contract=off tools/div_check.cpp -o /tmp/div_check
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rs = 0x1234567887654321ull;
static uint64_t rnd() {
    uint64_t z = (rs += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double rnd_d(int emin, int emax) {
    const uint64_t m = rnd() & 0xFFFFFFFFFFFFFull;
    const int e = emin + (int)(rnd() % (uint64_t)(emax - emin + 1));
    const uint64_t u = ((uint64_t)(e + 1023) << 52) | m;
    double x;
    memcpy(&x, &u, 8);
    return (rnd() & 1) ? -x : x;
}

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 20000000;
    long bad_r = 0, bad_q = 0, bad_q0 = 0;
    for (long i = 0; i < N; i++) {
        const double d = rnd_d(-60, 60);
        const double rn = 1.0 / d;
        double r0 = rn;
        const int mv = (int)(rnd() % 5) - 2;
        for (int k = 0; k < mv; k++) r0 = nextafter(r0, INFINITY);
        for (int k = 0; k > mv; k--) r0 = nextafter(r0, -INFINITY);
        const double r1 = fma(fma(-d, r0, 1.0), r0, r0);
        if (r1 != rn) { if (bad_r++ < 10) printf("rcp d=%a r0=%a r1=%a rn=%a\n", d, r0, r1, rn); }
        const double n = rnd_d(-60, 60);
        const double q0 = n * rn;
        const double q = fma(fma(-q0, d, n), rn, q0);
        if (q != n / d) { if (bad_q++ < 10) printf("div n=%a d=%a q=%a ieee=%a\n", n, d, q, n / d); }
        // the same with r0 (not correctly rounded): how often the quotient misrounds
        const double q0b = n * r0;
        const double qb = fma(fma(-q0b, d, n), r0, q0b);
        if (qb != n / d) bad_q0++;
    }
    printf("N=%ld: reciprocal step misses %ld, Markstein quotient (r = RN(1/d)) misses %ld, "
           "quotient with r within 2 ulp misses %ld\n", N, bad_r, bad_q, bad_q0);
    return (bad_r || bad_q) ? 1 : 0;
}

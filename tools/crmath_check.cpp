// crmath_check.cpp — host check of tools/crmath.h against glibc (the reference's libm).
// Build: g++ -O2 -mfma -ffp-contract=off -fno-builtin-sin -fno-builtin-cos tools/crmath_check.cpp -lm.
// For N random arguments per distribution it compares
//   ppcr::sincos(x)            with glibc sin(x), cos(x)
//   ppcr::atan2_refine(y, x, t0, ...) with glibc atan2(y, x) (t0 = glibc's value moved by -2..2 ulp,
//                              as the device's <= 1 ulp estimate would be), and the returned
//                              sin/cos with glibc sin/cos of the refined angle
// and writes every disagreement as "kind a b ours glibc" (%a) to stdout; the summary goes to
// stderr. tools/crmath_check.py decides each disagreement with mpmath at 200 bits.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "crmath.h"

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {   // splitmix64
    uint64_t z = (rs += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni() { return (double)(rnd() >> 11) * 0x1p-53; }

int main(int argc, char** argv) {
    const long N = argc > 1 ? atol(argv[1]) : 10000000;
    long bad_s = 0, bad_c = 0, bad_a = 0, bad_as = 0, bad_ac = 0, n_a = 0;
    for (long i = 0; i < N; i++) {
        // sin/cos: headings in [-pi, pi], degrees * pi / 180 over [-720, 720], small angles
        double x;
        switch (i % 3) {
            case 0: x = (2 * uni() - 1) * 3.141592653589793; break;
            case 1: x = ((2 * uni() - 1) * 720.0) * 3.141592653589793 / 180; break;
            default: x = (2 * uni() - 1) * ldexp(1.0, -(int)(rnd() % 40)); break;
        }
        double s, c;
        ppcr::sincos(x, s, c);
        if (s != sin(x)) { bad_s++; printf("sin %a 0 %a %a\n", x, s, sin(x)); }
        if (c != cos(x)) { bad_c++; printf("cos %a 0 %a %a\n", x, c, cos(x)); }
        // atan2 over step vectors: random directions and lengths (prev-path steps are 0..0.5 m),
        // plus near-axis directions
        double yy, xx;
        const double len = ldexp(uni() + 0.5, -(int)(rnd() % 8));
        if (i % 4 == 3) {
            const double th = (rnd() & 1 ? 0 : 1.5707963267948966) * (rnd() & 1 ? 1 : -1) + (2 * uni() - 1) * 1e-3;
            yy = len * sin(th); xx = len * cos(th);
        } else {
            const double th = (2 * uni() - 1) * 3.141592653589793;
            yy = len * sin(th); xx = len * cos(th);
        }
        if (yy == 0 || xx == 0) continue;
        n_a++;
        const double g = atan2(yy, xx);
        double t0 = g;
        const int mv = (int)(rnd() % 5) - 2;
        for (int k = 0; k < mv; k++) t0 = nextafter(t0, 10.0);
        for (int k = 0; k > mv; k--) t0 = nextafter(t0, -10.0);
        ppcr::dd S0, C0;
        ppcr::sincos_dd(t0, S0, C0);
        double as, ac;
        const double t = ppcr::atan2_refine(yy, xx, t0, S0, C0, as, ac);
        if (t != g) { bad_a++; printf("atan2 %a %a %a %a\n", yy, xx, t, g); }
        if (as != sin(t)) { bad_as++; printf("sin %a 0 %a %a\n", t, as, sin(t)); }
        if (ac != cos(t)) { bad_ac++; printf("cos %a 0 %a %a\n", t, ac, cos(t)); }
    }
    fprintf(stderr, "N=%ld: sin %ld, cos %ld differ; atan2 %ld of %ld differ; sin/cos(atan2) %ld/%ld differ\n",
            N, bad_s, bad_c, bad_a, n_a, bad_as, bad_ac);
    return 0;
}

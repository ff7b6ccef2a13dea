// pp_glibcm.h — sin, cos and atan2 exactly as the reference's libm computes them (host + device).
//
// The reference evaluates its trajectory frame with glibc's libm once per frame:
//   angle = atan2(pos_y - pos_y2, pos_x - pos_x2)           (src/main.cpp:607)
//   cos(-angle), sin(-angle), cos(angle), sin(angle)       (src/main.cpp:786-787, 822-823)
// and every spline knot, hence every point of every path, is a product with those values.
// glibc 2.35's sin/cos/atan2 are not correctly rounded: about 0.1 % of their results are the
// other neighbour of the exact value (tools/crmath_check.cpp + .py measure it against mpmath).
// Reproducing the reference bit for bit therefore needs glibc's own algorithms with glibc's own
// operation sequence. This header restates them for the variant the reference actually runs:
// the x86-64 FMA builds that glibc's ifunc selects on CPUs with FMA + AVX2 (__sin_fma,
// __cos_fma, __atan2_fma: sysdeps/ieee754/dbl-64/s_sin.c and e_atan2.c of glibc 2.35 compiled
// with -mfma -mavx2, so GCC contracted a*b + c into fused multiply-adds). Every fused
// multiply-add below is one the compiled library performs; every other operation is a plain
// IEEE double operation in the library's order. The data tables are the library's
// (pp_glibc_tables.h, tools/gen_glibc_tables.py). Checked: tests/test_glibcm.py (this header on
// the host == the system libm over millions of arguments) and the GPU test of the device build.
//
// Domain: sin/cos for |x| < 105414350 (glibc's reduce_sincos range; beyond it glibc uses a
// multi-word Payne-Hanek reduction not restated here: the functions return false and the caller
// keeps its own path, reachable only from an absurd telemetry yaw); atan2 everywhere.
// Rounding mode: round to nearest (glibc forces it around these functions).
#pragma once
#include <stdint.h>
#include <string.h>

#include "pp_glibc_tables.h"

#ifdef __HIPCC__
#define PPG_FN __host__ __device__ __forceinline__
#else
#define PPG_FN static inline
#endif

namespace ppg {

#if defined(__HIPCC__)
__constant__ double kSinCosTabD[440] = {PPG_SINCOSTAB_DATA};
__constant__ double kAtanTabD[241 * 7] = {PPG_ATANTAB_DATA};
#endif
static const double kSinCosTabH[440] = {PPG_SINCOSTAB_DATA};
static const double kAtanTabH[241 * 7] = {PPG_ATANTAB_DATA};

PPG_FN const double* sincostab() {
#if defined(__HIP_DEVICE_COMPILE__)
    return kSinCosTabD;
#else
    return kSinCosTabH;
#endif
}
PPG_FN const double* atantab() {
#if defined(__HIP_DEVICE_COMPILE__)
    return kAtanTabD;
#else
    return kAtanTabH;
#endif
}

PPG_FN double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
PPG_FN uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
PPG_FN double from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }
PPG_FN int32_t hi(double x) { return (int32_t)(bits(x) >> 32); }
PPG_FN uint32_t lo(double x) { return (uint32_t)bits(x); }
PPG_FN double fabs_(double x) { return from_bits(bits(x) & 0x7fffffffffffffffull); }
PPG_FN double copysign_(double x, double s) {
    return from_bits((bits(x) & 0x7fffffffffffffffull) | (bits(s) & 0x8000000000000000ull));
}

// ---- s_sin.c --------------------------------------------------------------------------------
constexpr double kSn3 = -0x1.5555555555515p-3, kSn5 = 0x1.11110e829872fp-7;
constexpr double kCs2 = 0x1p-1, kCs4 = -0x1.5555555555535p-5, kCs6 = 0x1.6c16bedd9e239p-10;
constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ecep-7, kS3 = -0x1.a01a019db08b8p-13,
                 kS4 = 0x1.71de27b9a7ed9p-19, kS5 = -0x1.addffc2fcdf59p-26;
constexpr double kBig = 0x1.8p45;                   // |x| + big rounds |x| to a multiple of 1/128
constexpr double kToint = 0x1.8p52, kHpinv = 0x1.45f306dc9c883p-1;
constexpr double kMp1 = 0x1.921fb58p0, kMp2 = -0x1.dde973cp-27, kPp3 = -0x1.cb3b398p-55,
                 kPp4 = -0x1.d747f23e32ed7p-83;
constexpr double kHp0 = 0x1.921fb54442d18p0, kHp1 = 0x1.1a62633145c07p-54;
constexpr double kTaylorMax = 0x1.020c49ba5e354p-3;   // 0.126

// TAYLOR_SIN(xx, a, da): sin(a + da) for |a| < 0.126
PPG_FN double taylor_sin(double xx, double a, double da) {
    double p = fma_(xx, kS5, kS4);
    p = fma_(xx, p, kS3);
    p = fma_(xx, p, kS2);
    p = fma_(xx, p, kS1);
    const double t1 = fma_(p, a, -(0.5 * da));
    const double t = fma_(xx, t1, da);
    return a + t;
}

// do_sin(x, dx) after the caller's sign rule (dx already negated where x <= 0): table path
PPG_FN double do_sin_tab(double x, double dx) {
    const double ax = fabs_(x);
    const double u = ax + kBig;
    const int k = (int)(lo(u) << 2);
    const double xr = ax - (u - kBig);
    const double xx = xr * xr;
    const double s = xr + fma_(xr * xx, fma_(xx, kSn5, kSn3), dx);
    const double c = fma_(xr, dx, xx * fma_(xx, fma_(xx, kCs6, kCs4), kCs2));
    const double* T = sincostab();
    const double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
    const double cor = fma_(s, cs, fma_(-c, sn, fma_(s, ccs, ssn)));
    return copysign_(sn + cor, x);
}

// do_cos(x, dx) after the caller's sign rule (dx negated where x < 0)
PPG_FN double do_cos_tab(double x, double dx) {
    const double ax = fabs_(x);
    const double u = ax + kBig;
    const int k = (int)(lo(u) << 2);
    const double xr = (ax - (u - kBig)) + dx;
    const double xx = xr * xr;
    const double s = fma_(xr * xx, fma_(xx, kSn5, kSn3), xr);
    const double c = xx * fma_(xx, fma_(xx, kCs6, kCs4), kCs2);
    const double* T = sincostab();
    const double sn = T[k], ssn = T[k + 1], cs = T[k + 2], ccs = T[k + 3];
    const double cor = fma_(-s, sn, fma_(-c, cs, fma_(-s, ssn, ccs)));
    return cs + cor;
}

// do_sin(a, da) as reached from the reductions: Taylor below 0.126, else the table with the
// sign rule "if (a <= 0) da = -da" (written !(0 < a) as the library tests it)
PPG_FN double do_sin(double a, double da) {
    if (fabs_(a) < kTaylorMax) return taylor_sin(a * a, a, da);
    if (!(0 < a)) da = -da;
    return do_sin_tab(a, da);
}
PPG_FN double do_cos(double a, double da) {
    if (a < 0) da = -da;
    return do_cos_tab(a, da);
}

// reduce_sincos: x = n pi/2 + a + da
PPG_FN int reduce(double x, double& a, double& da) {
    const double t = fma_(x, kHpinv, kToint);
    const double xn = t - kToint;
    const int n = (int)(lo(t) & 3);
    double y = fma_(-xn, kMp1, x);
    y = fma_(-xn, kMp2, y);
    const double t2 = fma_(-xn, kPp3, y);
    double db = fma_(-kPp3, xn, y - t2);
    const double b = fma_(-xn, kPp4, t2);
    db = db + fma_(-xn, kPp4, t2 - b);
    a = b;
    da = db;
    return n;
}

// sin(x): glibc's __sin for |x| < 105414350; false (s untouched) beyond, and for inf/NaN
PPG_FN bool sin(double x, double& s) {
    const int32_t k = hi(x) & 0x7fffffff;
    if (k < 0x3e500000) { s = x; return true; }                       // |x| < 2^-26
    if (k < 0x3feb6000) {                                               // |x| < 0.855469
        if (fabs_(x) < kTaylorMax) { s = taylor_sin(x * x, x, 0.0); return true; }
        s = do_sin_tab(x, (x > 0) ? 0.0 : -0.0);
        return true;
    }
    if (k < 0x400368fd) {                                               // |x| < 2.426265
        const double t = kHp0 - fabs_(x);
        const double dx = (t < 0) ? -kHp1 : kHp1;
        s = copysign_(do_cos_tab(t, dx), x);
        return true;
    }
    if (k < 0x419921fb) {                                               // |x| < 105414350
        double a, da;
        const int n = reduce(x, a, da);
        double r = (n & 1) ? do_cos(a, da) : do_sin(a, da);
        s = (n & 2) ? -r : r;
        return true;
    }
    return false;
}

// cos(x): glibc's __cos, same domain
PPG_FN bool cos(double x, double& c) {
    const int32_t k = hi(x) & 0x7fffffff;
    if (k < 0x3e400000) { c = 1.0; return true; }                     // |x| < 2^-27
    if (k < 0x3feb6000) {                                               // |x| < 0.855469
        c = do_cos_tab(x, (x < 0) ? -0.0 : 0.0);
        return true;
    }
    if (k < 0x400368fd) {                                               // |x| < 2.426265
        const double y = kHp0 - fabs_(x);
        const double a = y + kHp1;
        const double da = (y - a) + kHp1;
        c = do_sin(a, da);
        return true;
    }
    if (k < 0x419921fb) {
        double a, da;
        const int n = reduce(x, a, da);
        double r = (n & 1) ? do_sin(a, da) : do_cos(a, da);
        c = ((n + 1) & 2) ? -r : r;
        return true;
    }
    return false;
}

// ---- e_atan2.c (glibc 2.35, after the removal of the multi-precision paths) ----------------
constexpr double kPi = 0x1.921fb54442d18p1, kPiLo = 0x1.1a62633145c07p-53;
constexpr double kPio2 = 0x1.921fb54442d18p0, kPio2Lo = 0x1.1a62633145c07p-54;
constexpr double kPio4 = 0x1.921fb54442d18p-1, k3Pio4 = 0x1.2d97c7f3321d2p1;
constexpr double kA1 = 0x1.375f08b31cbcep-4, kA2 = -0x1.7458022b13c25p-4, kA3 = 0x1.c71c6e5129a3bp-4,
                 kA4 = -0x1.24924923f7603p-3, kA5 = 0x1.99999999997fdp-3, kA6 = -0x1.5555555555555p-2;

// A6 + v (A5 + v (A4 + ...)), v = u^2: atan(u) = u + u^3 (this) below 1/16
PPG_FN double atan_series(double v) {
    double p = fma_(v, kA1, kA2);
    p = fma_(v, p, kA3);
    p = fma_(v, p, kA4);
    p = fma_(v, p, kA5);
    return fma_(v, p, kA6);
}
// the table entry of u in [1/16, 1]: index round(u * 256) - 16
PPG_FN const double* atan_entry(double u) {
    const double t = fma_(u, 256.0, 0x1p52) - 0x1p52;
    return atantab() + 7 * ((int)t - 16);
}
// e2 + v (e3 + v (e4 + v (e5 + v e6)))
PPG_FN double atan_tab_poly(const double* e, double v) {
    double p = fma_(v, e[6], e[5]);
    p = fma_(v, p, e[4]);
    p = fma_(v, p, e[3]);
    return fma_(v, p, e[2]);
}

PPG_FN double atan2(double y, double x) {
    const int32_t hx = hi(x), hy = hi(y);
    const uint32_t lx = lo(x), ly = lo(y);
    if ((hx & 0x7ff00000) == 0x7ff00000 && ((hx & 0xfffff) | lx)) return x + y;    // x NaN
    if ((hy & 0x7ff00000) == 0x7ff00000 && ((hy & 0xfffff) | ly)) return y + y;    // y NaN
    if (hy == 0) {                                                    // y = +0 or tiny positive
        if (ly == 0) return hx < 0 ? kPi : 0.0;
        if (x == 0) return kPio2;
    } else {
        if (ly == 0 && (uint32_t)hy == 0x80000000u) return hx < 0 ? -kPi : -0.0;   // y = -0
        if (x == 0) return hy < 0 ? -kPio2 : kPio2;
    }
    if (hx == 0x7ff00000 && lx == 0) {                               // x = +inf
        if (hy == 0x7ff00000) return kPio4;
        if ((uint32_t)hy == 0xfff00000u) return -kPio4;
        return hy < 0 ? -0.0 : 0.0;
    }
    if (lx == 0 && (uint32_t)hx == 0xfff00000u) {                    // x = -inf
        if (hy == 0x7ff00000) return k3Pio4;
        if ((uint32_t)hy == 0xfff00000u) return -k3Pio4;
        return hy < 0 ? -kPi : kPi;
    }
    if (hy == 0x7ff00000 && ly == 0) return kPio2;                    // y = +inf
    if ((uint32_t)hy == 0xfff00000u && ly == 0) return -kPio2;       // y = -inf
    const int32_t ediff = (hy & 0x7ff00000) - (hx & 0x7ff00000);
    double ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
    if (ediff > 0x38fffff) return (0 < y) ? kPio2 : -kPio2;          // |y/x| > 2^56
    if (ediff < -0x38fffff) {                                         // |y/x| < 2^-56
        if (x > 0) return copysign_(ay / ax, y);
        return (0 < y) ? kPi : -kPi;
    }
    // moderate ratio: scale both away from the exponent range's ends
    if (0x1p-500 > ax || 0x1p-500 > ay) { ax *= 0x1p500; ay *= 0x1p500; }
    if (ax > 0x1p500 || ay > 0x1p500) { ax *= 0x1p-500; ay *= 0x1p-500; }
    // u = the smaller over the larger magnitude, du its remainder (the product's error by fma)
    const bool xbig = ax > ay;
    const double num = xbig ? ay : ax, den = xbig ? ax : ay;
    const double u = num / den;
    const double pr = den * u;
    const double du = ((num - pr) - fma_(den, u, -pr)) / den;
    double res;
    if (x > 0) {
        if (xbig) {                                                   // atan(u)
            if (u < 0.0625) {
                const double v = u * u;
                res = u + fma_(u * v, atan_series(v), du);
            } else {
                const double* e = atan_entry(u);
                const double vv = u - e[0];
                const double v1 = du + vv;
                const double dv = (fabs_(vv) > fabs_(du)) ? (vv - v1) + du : (du - v1) + vv;
                double q = fma_(v1, e[6], e[5]);
                q = fma_(v1, q, e[4]);
                q = fma_(v1, q, e[3]);
                q = (v1 * v1) * q;
                q = fma_(dv, e[2], q);
                res = fma_(v1, e[2], q) + e[1];
            }
        } else {                                                      // pi/2 - atan(u)
            if (u < 0.0625) {
                const double v = u * u;
                const double w = (u * v) * atan_series(v);
                const double t = kPio2 - u;
                double r = (kPio2 > fabs_(u)) ? (kPio2 - t) - u : kPio2 - (u + t);
                r = r + kPio2Lo;
                r = r - du;
                r = r - w;
                res = r + t;
            } else {
                const double* e = atan_entry(u);
                const double v1 = (u - e[0]) + du;
                res = (kPio2 - e[1]) + fma_(-v1, atan_tab_poly(e, v1), kPio2Lo);
            }
        }
    } else if (!(ay > ax)) {                                          // pi - atan(u)
        if (u < 0.0625) {
            const double v = u * u;
            const double w = (v * u) * atan_series(v);
            const double t = kPi - u;
            double r = (kPi > fabs_(u)) ? (kPi - t) - u : kPi - (t + u);
            r = r + kPiLo;
            r = r - du;
            r = r - w;
            res = r + t;
        } else {
            const double* e = atan_entry(u);
            const double v1 = (u - e[0]) + du;
            res = (kPi - e[1]) + fma_(-v1, atan_tab_poly(e, v1), kPiLo);
        }
    } else {                                                          // pi/2 + atan(u)
        if (u < 0.0625) {
            const double v = u * u;
            const double w = (v * u) * atan_series(v);
            const double t = u + kPio2;
            double r = (kPio2 > fabs_(u)) ? (kPio2 - t) + u : (u - t) + kPio2;
            r = r + kPio2Lo;
            r = r + du;
            r = r + w;
            res = r + t;
        } else {
            const double* e = atan_entry(u);
            const double v1 = (u - e[0]) + du;
            res = (kPio2 + e[1]) + fma_(v1, atan_tab_poly(e, v1), kPio2Lo);
        }
    }
    return copysign_(res, y);
}

}  // namespace ppg

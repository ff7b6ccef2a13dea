// pp_math.h — register-light FP64 transcendentals for the candidate loop (gfx950).
//
// The ROCm device library's f64 sin/cos carry the large-argument (Payne-Hanek) reduction inline and
// atan2 a wide argument-reduction tree: together ~80 VGPRs of the loop's register peak (measured
// with -Rpass-analysis=kernel-resource-usage), which halves occupancy. The planner only feeds them
// small arguments (headings and turn angles), so these are the classic fdlibm-style algorithms
// (Cody-Waite reduction by pi/2, minimax kernels, atan with 4-interval reduction), < 1 ulp like
// glibc's, with the rare large-argument case handed to the device library in a non-inlined call.
// All arithmetic is plain IEEE double (the library is built with -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ppm {

// a * b + c as the three-address v_fma_f64. The compiler lowers __builtin_fma with a register
// addend that stays live (a loop-invariant polynomial coefficient) to v_mov_b64 + the two-address
// v_fmac_f64, one extra issue per term; PP_FMA3=0 keeps __builtin_fma.
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__device__ __forceinline__ int hiword(double x) { return (int)(__double_as_longlong(x) >> 32); }
__device__ __forceinline__ unsigned loword(double x) { return (unsigned)__double_as_longlong(x); }
__device__ __forceinline__ double from_words(int hi, unsigned lo) {
    return __longlong_as_double(((long long)hi << 32) | (long long)lo);
}

// ---- sin / cos kernels on [-pi/4, pi/4] with tail y (x + y = reduced argument) -------------
__device__ __forceinline__ double ksin(double x, double y, bool has_tail) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const int ix = hiword(x) & 0x7fffffff;
    if (ix < 0x3e400000) return x;                 // |x| < 2^-27
    const double z = x * x;
    const double v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (!has_tail) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

__device__ __forceinline__ double kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const int ix = hiword(x) & 0x7fffffff;
    if (ix < 0x3e400000) return 1.0;               // |x| < 2^-27
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));   // |x| < 0.3
    const double qx = (ix > 0x3fe90000) ? 0.28125 : from_words(ix - 0x00200000, 0u);
    const double hz = 0.5 * z - qx;
    const double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

__device__ __attribute__((noinline)) void sincos_large(double x, double* s, double* c) {
    *s = sin(x);
    *c = cos(x);
}

// sin and cos of x. Medium-size Cody-Waite reduction (3-part pi/2) for |x| <= 2^19 * pi/2;
// beyond that the device library's reduction — compiled in only when kLarge (the hot loop is
// instantiated without it: its arguments are bounded, see kSlowAngle in pp_eval.hip).
constexpr double kMediumMax = 823549.6;   // < 2^19 * pi/2 (high word 0x413921fb)
template <bool kLarge = true>
__device__ __forceinline__ void sincos_pp(double x, double& s, double& c) {
    const int hx = hiword(x);
    const int ix = hx & 0x7fffffff;
    if (ix <= 0x3fe921fb) {                         // |x| <= pi/4
        s = ksin(x, 0.0, false);
        c = kcos(x, 0.0);
        return;
    }
    if (ix > 0x413921fb) {                          // huge, inf or NaN
        if (kLarge) {
            sincos_large(x, &s, &c);
        } else {
            s = c = __builtin_nan("");                 // unreachable by construction
        }
        return;
    }
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    double t = fabs(x);
    const int n = (int)(t * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t - fn * pio2_1;
    double w = fn * pio2_1t;                        // first round good to 85 bits
    const int j = ix >> 20;
    double y0 = r - w;
    int i = j - ((hiword(y0) >> 20) & 0x7ff);
    if (i > 16) {                                   // cancellation: second round, 118 bits
        t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y0 = r - w;
        i = j - ((hiword(y0) >> 20) & 0x7ff);
        if (i > 49) {                               // third round, 151 bits
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y0 = r - w;
        }
    }
    double y1 = (r - y0) - w;
    int q = n;
    if (hx < 0) { y0 = -y0; y1 = -y1; q = -n; }
    const double ks = ksin(y0, y1, true);
    const double kc = kcos(y0, y1);
    switch (q & 3) {
        case 0: s = ks; c = kc; break;
        case 1: s = kc; c = -ks; break;
        case 2: s = -ks; c = -kc; break;
        default: s = -kc; c = ks; break;
    }
}

// ---- atan / atan2 --------------------------------------------------------------------------
__device__ __forceinline__ double atan_pos(double x, int ix) {
    // x >= 0, ix = high word of x; |x| < 2^66
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    int id;
    double hi = 0, lo = 0;
    if (ix < 0x3fdc0000) {                          // |x| < 0.4375
        if (ix < 0x3e400000) return x;              // |x| < 2^-27
        id = -1;
    } else if (ix < 0x3ff30000) {                   // |x| < 1.1875
        if (ix < 0x3fe60000) {                      // 7/16 <= |x| < 11/16
            id = 0; hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17;
            x = (2.0 * x - 1.0) / (2.0 + x);
        } else {                                    // 11/16 <= |x| < 19/16
            id = 1; hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17;
            x = (x - 1.0) / (x + 1.0);
        }
    } else if (ix < 0x40038000) {                   // |x| < 2.4375
        id = 2; hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17;
        x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {                                        // 2.4375 <= |x| < 2^66
        id = 3; hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17;
        x = -1.0 / x;
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    return hi - ((x * (s1 + s2) - lo) - x);
}

// atan2 for zero / infinite / NaN arguments (C standard Annex F values)
__device__ __forceinline__ double atan2_special(double y, double x) {
    const double pi = 3.1415926535897931160E+00, pi_o_2 = 1.5707963267948965580E+00,
                 pi_o_4 = 7.8539816339744827900E-01;
    if (x != x || y != y) return x + y;
    const bool xneg = hiword(x) < 0;
    const double sy = hiword(y) < 0 ? -1.0 : 1.0;
    if (y == 0.0) return xneg ? sy * pi : y;                    // atan2(+-0, x)
    const bool xinf = fabs(x) == __builtin_inf(), yinf = fabs(y) == __builtin_inf();
    if (yinf && xinf) return xneg ? sy * 3.0 * pi_o_4 : sy * pi_o_4;
    if (yinf || x == 0.0) return sy * pi_o_2;
    return xneg ? sy * pi : sy * 0.0;                            // x = +-inf, y finite
}

// atan2(y, x): quadrant logic of the C standard; finite nonzero arguments take the fast path.
__device__ __forceinline__ double atan2_pp(double y, double x) {
    const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16,
                 pi_o_2 = 1.5707963267948965580E+00;
    const int hx = hiword(x), hy = hiword(y);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const bool x_special = (ix | loword(x)) == 0 || ix >= 0x7ff00000;
    const bool y_special = (iy | loword(y)) == 0 || iy >= 0x7ff00000;
    if (x_special || y_special) return atan2_special(y, x);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2*sign(x) + sign(y)
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) {
        z = pi_o_2 + 0.5 * pi_lo;                    // |y/x| > 2^60
    } else if (hx < 0 && k < -60) {
        z = 0.0;                                     // |y|/x < -2^60
    } else {
        const double q = fabs(y / x);
        z = atan_pos(q, hiword(q));
    }
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// Branch-free atan2 for finite nonzero (y, x): ONE division and no divergent interval branches.
// The argument reduction of atan_pos is applied to (|y|, |x|) directly — e.g. t = (|y|-|x|) /
// (|x|+|y|) instead of (q-1)/(q+1) with a rounded q = |y|/|x| — so the reduced argument carries a
// single rounding (slightly more accurate than the two-division form). Interval selection by
// exact comparisons of |y| against 7/16, 11/16, 19/16, 39/16 times |x| (scaled by 16, exact in
// double for the magnitudes that reach this path); the quadrant logic is atan2_pp's.
__device__ __forceinline__ double atan2_fast(double y, double x) {
    const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    const int hx = hiword(x), hy = hiword(y);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const bool x_special = (ix | loword(x)) == 0 || ix >= 0x7ff00000;
    const bool y_special = (iy | loword(y)) == 0 || iy >= 0x7ff00000;
    const int k = (iy - ix) >> 20;
    if (__builtin_expect(x_special || y_special || k > 60 || k < -60, 0)) return atan2_pp(y, x);
    const double ay = fabs(y), ax = fabs(x);
    const double y16 = 16.0 * ay;
    // interval id: -1 (q < 7/16), 0 (< 11/16), 1 (< 19/16), 2 (< 39/16), 3 (>= 39/16)
    const int id = (y16 < 7.0 * ax) ? -1 : (y16 < 11.0 * ax) ? 0 : (y16 < 19.0 * ax) ? 1
                 : (y16 < 39.0 * ax) ? 2 : 3;
    // t = num / den per interval (fdlibm's reductions multiplied through by |x|)
    double num, den, hi, lo;
    if (id < 0)       { num = ay;                  den = ax;                  hi = 0.0; lo = 0.0; }
    else if (id == 0) { num = 2.0 * ay - ax;       den = 2.0 * ax + ay;
                        hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
    else if (id == 1) { num = ay - ax;             den = ax + ay;
                        hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
    else if (id == 2) { num = 2.0 * ay - 3.0 * ax; den = 2.0 * ax + 3.0 * ay;
                        hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
    else              { num = -ax;                 den = ay;
                        hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
    const double t = num / den;
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const double z = t * t;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const double zz = (id < 0) ? t - t * (s1 + s2) : hi - ((t * (s1 + s2) - lo) - t);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2*sign(x) + sign(y)
    return m == 0 ? zz : m == 1 ? -zz : m == 2 ? pi - (zz - pi_lo) : (zz - pi_lo) - pi;
}

// atan2_fast for finite (y, x) that are not both zero (the wide-turn branch of the candidate
// loop: components of unit vectors): no special-case fallback. Zero, tiny (|y/x| < 2^-60) and huge
// (> 2^60) ratios go through the same reduction: t = 0 or a tiny/huge-ratio t gives the values
// atan2_pp returns for them (+-0, +-pi/2, +-pi: hi + lo and pi - (t - pi_lo) round to those
// constants), NaN propagates. tools/atan2_check.hip compares the two on the GPU.
// atan_pos's interval constants (hi, lo) for id = -1 .. 3 (atan2_unit)
__constant__ double kAtanHiLo[10] = {
    0.0, 0.0,
    4.63647609000806093515e-01, 2.26987774529616870924e-17,
    7.85398163397448278999e-01, 3.06161699786838301793e-17,
    9.82793723247329054082e-01, 1.39033110312309984516e-17,
    1.57079632679489655800e+00, 6.12323399573676603587e-17};
__device__ __forceinline__ double atan2_unit(double y, double x) {
    const double pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    const int hy = hiword(y);
    const double ay = fabs(y), ax = fabs(x);
    const double y16 = 16.0 * ay;
    const int id = (y16 < 7.0 * ax) ? -1 : (y16 < 11.0 * ax) ? 0 : (y16 < 19.0 * ax) ? 1
                 : (y16 < 39.0 * ax) ? 2 : 3;
    double num, den;
    if (id < 0)       { num = ay;                  den = ax; }
    else if (id == 0) { num = 2.0 * ay - ax;       den = 2.0 * ax + ay; }
    else if (id == 1) { num = ay - ax;             den = ax + ay; }
    else if (id == 2) { num = 2.0 * ay - 3.0 * ax; den = 2.0 * ax + 3.0 * ay; }
    else              { num = -ax;                 den = ay; }
    // the interval constants by a per-lane table load: the branch is rare, and constants
    // selected in registers would be hoisted out of the candidate loop and held there
    const double hi = kAtanHiLo[2 * (id + 1)], lo = kAtanHiLo[2 * (id + 1) + 1];
    const double t = num / den;
    const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
                 aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
                 aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
                 aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
                 aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
                 aT10 = 1.62858201153657823623e-02;
    const double z = t * t;
    const double w = z * z;
    const double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const double zz = (id < 0) ? t - t * (s1 + s2) : hi - ((t * (s1 + s2) - lo) - t);
    const int m = ((hy >> 31) & 1) | (x < 0.0 ? 2 : 0);   // x = -0 counts as +0 (atan2(y, -0) = +-pi/2)
    return m == 0 ? zz : m == 1 ? -zz : m == 2 ? pi - (zz - pi_lo) : (zz - pi_lo) - pi;
}

// Angle between consecutive step directions without atan2 (run_candidate). The reference turns
// each step (dx, dy) into an absolute angle atan2(dy, dx) and wraps the difference to the previous
// one (src/main.cpp:934). For unit vectors u_prev, u the signed angle is asin(u_prev x u) while
// u_prev . u > 0 and |u_prev x u| <= kStepSinMax (|angle| <= 0.0708 rad): the Taylor series through
// s^13 is then accurate to ~1e-18 relative (next term c7 s^15 < 1.1e-18 s), and the unit vectors
// carry ~2 ulp, so the angle differs from atan2(dy,dx) - atan2(dy',dx') by < 1e-17 rad. The caller
// applies the reference's wrap fmod(. + 3 pi, 2 pi) - pi to it, whose rounding grid (ulp(3 pi) =
// 1.8e-15) dominates, exactly as it does for the reference's own difference of two atan2 values.
constexpr double kStepSinMax = 0.0708;
__device__ __forceinline__ double asin_small(double s) {
    const double c1 = 1.66666666666666666667e-01, c2 = 7.50000000000000000000e-02,
                 c3 = 4.46428571428571428571e-02, c4 = 3.03819444444444444444e-02,
                 c5 = 2.23721590909090909091e-02, c6 = 1.73527644230769230769e-02;
    const double z = s * s;
    double p = fma3(z, c6, c5);
    p = fma3(z, p, c4);
    p = fma3(z, p, c3);
    p = fma3(z, p, c2);
    p = fma3(z, p, c1);
    return __builtin_fma(s * z, p, s);
}
// asin_small with its coefficients materialised in scalar registers at the use (PP_ASIN_S): the
// loop then holds no coefficient in vector registers (12 VGPRs), at one v_mov_b64 for the first
// term (a VOP3 reads one scalar operand)
__device__ __forceinline__ double kcs(double v) {
    asm volatile("" : "+s"(v));
    return v;
}
__device__ __forceinline__ double fma_vvs(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
// the same with compiler-visible fused multiply-adds and constants (no inline-asm hazard padding)
__device__ __forceinline__ double asin_small_b(double s) {
    const double z = s * s;
    double p = __builtin_fma(z, 1.73527644230769230769e-02, 2.23721590909090909091e-02);
    p = __builtin_fma(z, p, 3.03819444444444444444e-02);
    p = __builtin_fma(z, p, 4.46428571428571428571e-02);
    p = __builtin_fma(z, p, 7.50000000000000000000e-02);
    p = __builtin_fma(z, p, 1.66666666666666666667e-01);
    return __builtin_fma(s * z, p, s);
}
__device__ __forceinline__ double asin_small_s(double s) {
    const double z = s * s;
    double c6 = kcs(1.73527644230769230769e-02);
    asm volatile("" : "+v"(c6));
    double p = fma_vvs(z, c6, kcs(2.23721590909090909091e-02));
    p = fma_vvs(z, p, kcs(3.03819444444444444444e-02));
    p = fma_vvs(z, p, kcs(4.46428571428571428571e-02));
    p = fma_vvs(z, p, kcs(7.50000000000000000000e-02));
    p = fma_vvs(z, p, kcs(1.66666666666666666667e-01));
    return __builtin_fma(s * z, p, s);
}

// 1/d to ~1 ulp: v_rcp_f64 and two Newton steps (d finite, normal)
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    return r;
}

// 1/d to ~2^-48 relative: v_rcp_f64 (~2^-24: tools/rcp_check.hip) and one Newton step. Enough for
// the Markstein quotient below: with r = (1 + e)/d its result carries ~e^2 = 2^-96 of relative error
// before the final rounding, which is therefore the correct one (a quotient within 2^-96 of a
// rounding midpoint is the only exception), exactly as with rcp_nr's r
__device__ __forceinline__ double rcp_nr1(double d) {
    const double r = __builtin_amdgcn_rcp(d);
    return __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
}

// n / d from r ~ 1/d (within ~1 ulp): q0 = n r, then one Markstein correction with the exact
// residual n - q0 d (fma). With r within half an ulp of 1/d (r = RN(1/d), e.g. 0.02 for 50) the
// result is the correctly rounded quotient; with rcp_nr's r it is in all but rare cases (then one
// ulp away). Zero and non-finite operands, and |d| or |n| outside [2^-900, 2^900] (where the
// residual could underflow), take the IEEE division.
__device__ __forceinline__ double div_rcp(double n, double d, double r) {
    const double q0 = n * r;
    const double e = __builtin_fma(-q0, d, n);
    const double q = __builtin_fma(e, r, q0);
    const double ad = fabs(d), an = fabs(n);
    const bool ok = ad >= 0x1p-900 && ad <= 0x1p900 && (an == 0.0 || (an >= 0x1p-900 && an <= 0x1p900));
    if (__builtin_expect(!ok, 0)) return n / d;
    return an == 0.0 ? q0 : q;        // +-0 / d: q0 carries the quotient's sign
}

// div_rcp without its range checks, for operands known to stay in range: the caller's
// k_cand<false> instantiation runs only scenes whose speeds and ramp times k_prep checked
// (kLimSlow otherwise). The sign of a zero quotient may differ from the IEEE one.
__device__ __forceinline__ double div_rcp_nc(double n, double d, double r) {
    const double q0 = n * r;
    return __builtin_fma(__builtin_fma(-q0, d, n), r, q0);
}

// div_rcp_nc(v, 50, 0.02) with the residual fma written three-address (v stays live after it, so
// the compiler's two-address v_fmac would need a copy of v first); 50 from an SGPR pair
__device__ __forceinline__ double div50_nc(double v) {
    const double q0 = v * 0.02;
    double e;
    asm("v_fma_f64 %0, -%1, %2, %3" : "=v"(e) : "v"(q0), "s"(50.0), "v"(v));
    return __builtin_fma(e, 0.02, q0);
}

// n / d with r ~ 1/d for a d known to lie in [2^-450, 2^450] (dok: sqrt_rd's fast path);
// otherwise, and for |n| outside [2^-900, 2^900], the IEEE division
__device__ __forceinline__ double div_rcp_n(double n, double d, double r, bool dok) {
    const double q0 = n * r;
    const double e = __builtin_fma(-q0, d, n);
    const double q = __builtin_fma(e, r, q0);
    const double an = fabs(n);
    if (__builtin_expect(!(dok && an >= 0x1p-900 && an <= 0x1p900), 0)) return (dok && an == 0.0) ? q0 : n / d;
    return q;
}

// div_rcp_n for k_cand<false>: the numerators (x - pos_x) dstep and (y - pos_y) dstep with dstep
// +0 or in [2^-119, 2^15] stay below 2^900, and a numerator below 2^-900 (a step of ~1e-150 m and
// less) may take an ulp of error only at that scale; so only d's range (dok) picks the IEEE
// division. n = +-0 gives q0 = +-0 and a zero correction, as the IEEE quotient.
__device__ __forceinline__ double div_rcp_d(double n, double d, double r, bool dok) {
    const double q0 = n * r;
    const double q = __builtin_fma(__builtin_fma(-q0, d, n), r, q0);
    if (__builtin_expect(!dok, 0)) return n / d;
    return q;
}

// d = sqrt(q) correctly rounded and rd ~ 1/d; returns whether q was in [2^-900, 2^900]. There
// this is the ISA sequence the compiler emits for an IEEE sqrt (v_rsq_f64, then Goldschmidt
// g ~ sqrt(q), h ~ 1/(2 sqrt(q)) and two residual corrections of g), without its range scaling
// and 0/inf fix-ups, and rd = 2 h. Elsewhere (0, tiny, huge, inf, NaN): sqrt and 1 / d.
__device__ __forceinline__ bool sqrt_rd(double q, double& d, double& rd) {
    if (__builtin_expect(q >= 0x1p-900 && q <= 0x1p900, 1)) {
        const double y0 = __builtin_amdgcn_rsq(q);
        double g = q * y0;
        double h = 0.5 * y0;
        const double e = __builtin_fma(-h, g, 0.5);
        g = __builtin_fma(g, e, g);
        h = __builtin_fma(h, e, h);
        const double d0 = __builtin_fma(-g, g, q);
        g = __builtin_fma(d0, h, g);
        const double d1 = __builtin_fma(-g, g, q);
        d = __builtin_fma(d1, h, g);
        rd = 2.0 * h;
        return true;
    }
#ifdef PP_CENSUS
    asm volatile(";@R 9 sqrtslow");      // (tools/valu_census.py region marker)
#endif
    d = __builtin_sqrt(q);
    rd = 1.0 / d;
    return false;
}

// fmod(a, 2*pi) for the reference's angle wrap fmod(d + 3*pi, 2*pi) - pi
// (src/main.cpp:870, 934). fmod is exact, so any exact evaluation is bit-identical: for
// 0 <= a < 3*(2*pi) the remainder a - k*(2*pi), k in {0, 1, 2}, is computed exactly
// (Sterbenz: y <= a < 4y for the k = 2 case, with 2y and 3y exact doubles). Other finite inputs
// are reduced by exact subtractions of y * 2^j (each r - y*2^j with y*2^j <= r < y*2^(j+1) is
// exact by Sterbenz), the textbook long division fmod performs.
// fmod_2pi for a in [0, 3 * 2pi) or NaN (a = atan2 + 3 pi): its first three cases; NaN - 2y = NaN
__device__ __forceinline__ double fmod_2pi_small(double a) {
    const double y = 2 * 3.14159265358979323846;
    if (a < y) return a;
    if (a < 2.0 * y) return a - y;
    return a - 2.0 * y;
}
__device__ __forceinline__ double fmod_2pi(double a) {
    const double y = 2 * 3.14159265358979323846;
    if (a >= 0.0 && a < y) return a;
    if (a >= y && a < 2.0 * y) return a - y;
    if (a >= 2.0 * y && a < 3.0 * y) return a - 2.0 * y;
    if (!(fabs(a) < __builtin_inf())) return a - a;   // inf, NaN -> NaN
    double r = fabs(a);
    while (r >= y) {
        double t = y;
        while (t * 2.0 <= r) t *= 2.0;
        r -= t;
    }
    return a < 0 ? -r : r;
}

}  // namespace ppm

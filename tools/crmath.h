// crmath.h — correctly rounded sin, cos and atan2 (double-double evaluation): a measuring tool.
//
// The reference computes the trajectory frame once per frame with glibc's libm:
//   angle = atan2(pos_y - pos_y2, pos_x - pos_x2)           (src/main.cpp:607)
//   cos(-angle), sin(-angle), cos(angle), sin(angle)       (src/main.cpp:786-787, 822-823)
// and every knot of the spline (hence every point of every candidate path) is a product with
// those four values. glibc 2.35's sin/cos/atan2 (IBM Accurate Mathematical Library lineage)
// return the correctly rounded result for all but a vanishing fraction of arguments
// (tools/crmath_check.cpp measures it against mpmath on the planner's argument ranges), so
// reproducing the reference's frame bit for bit needs correctly rounded functions, not merely
// faithful (<= 1 ulp) ones: one ulp in cos(angle) moves the knots by an ulp, and decisions that
// test exact equality downstream (the standstill step dist == 0 at src/main.cpp:1025) follow it.
//
// Method: argument reduction by pi/2 in four parts (three 33-bit parts, so n * P_i is exact for
// n < 2^20, and a 53-bit tail), Taylor series of sin and cos on |r| <= pi/4 in double-double
// (relative error ~2^-100), one rounding at the end. atan2: the <= 1 ulp fdlibm-style value t0
// (ppm::atan2_pp) is corrected by atan(delta) ~= delta, delta = (y cos t0 - x sin t0) /
// (x cos t0 + y sin t0), with cos/sin t0 in double-double; the heading's sin/cos are then those
// of the rounded angle by a first-order Taylor step from t0. These run once per scene in k_prep.
// Requires |x| < kCrMax for sin/cos (the medium reduction range); callers keep larger arguments
// on the non-CR path (only reachable from an absurd telemetry yaw).
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define PPCR_FN __host__ __device__ __forceinline__
#else
#define PPCR_FN static inline
#endif

namespace ppcr {

struct dd { double h, l; };

constexpr double kCrMax = 823549.6;        // < 2^19 * pi/2: n < 2^20 in the reduction

PPCR_FN uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
PPCR_FN double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

PPCR_FN dd two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
PPCR_FN dd fast_two_sum(double a, double b) {   // |a| >= |b| (or a == 0)
    const double s = a + b;
    return {s, b - (s - a)};
}
PPCR_FN dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma_(a, b, -p)};
}
PPCR_FN dd add(dd a, dd b) {
    dd s = two_sum(a.h, b.h);
    const dd t = two_sum(a.l, b.l);
    s.l += t.h;
    s = fast_two_sum(s.h, s.l);
    s.l += t.l;
    return fast_two_sum(s.h, s.l);
}
PPCR_FN dd mul(dd a, dd b) {
    dd p = two_prod(a.h, b.h);
    p.l = fma_(a.h, b.l, p.l);
    p.l = fma_(a.l, b.h, p.l);
    return fast_two_sum(p.h, p.l);
}
PPCR_FN dd neg(dd a) { return {-a.h, -a.l}; }

// (-1)^k / (2k+1)!, k = 1..13 and (-1)^k / (2k)!, k = 1..14 (tools/gen_crmath_consts.py)
constexpr double kSinH[13] = {-0.16666666666666666, 0.008333333333333333, -0.0001984126984126984,
    2.7557319223985893e-06, -2.505210838544172e-08, 1.6059043836821613e-10, -7.647163731819816e-13,
    2.8114572543455206e-15, -8.22063524662433e-18, 1.9572941063391263e-20, -3.868170170630684e-23,
    6.446950284384474e-26, -9.183689863795546e-29};
constexpr double kSinL[13] = {-9.25185853854297e-18, 1.1564823173178714e-19, -1.7209558293420705e-22,
    -1.858393274046472e-22, 1.448814070935912e-24, 1.2585294588752098e-26, -7.03872877733453e-30,
    1.6508842730861433e-31, -2.2141894119604265e-34, -1.3643503830087908e-36, 8.843177655482344e-40,
    -1.9330404233703465e-42, -1.4303150396787322e-45};
constexpr double kCosH[14] = {-0.5, 0.041666666666666664, -0.001388888888888889, 2.48015873015873e-05,
    -2.755731922398589e-07, 2.08767569878681e-09, -1.1470745597729725e-11, 4.779477332387385e-14,
    -1.5619206968586225e-16, 4.110317623312165e-19, -8.896791392450574e-22, 1.6117375710961184e-24,
    -2.4795962632247976e-27, 3.279889237069838e-30};
constexpr double kCosL[14] = {0.0, 2.3129646346357427e-18, 5.300543954373577e-20, 2.1511947866775882e-23,
    -2.3767714622250297e-23, -1.20734505911326e-25, -2.0655512752830745e-28, 4.399205485834081e-31,
    -1.1910679660273754e-32, 1.4412973378659527e-36, 7.911402614872376e-38, -3.6846573564509766e-41,
    1.2953730964765229e-43, 1.5117542744029879e-46};
// pi/2 = P1 + P2 + P3 + P4 (P1..P3: 33 significant bits each), residual 7.4e-49
constexpr double kP1 = 1.5707963267341256, kP2 = 6.077100506303966e-11, kP3 = 2.0222662487111665e-21,
                 kP4 = 8.4784276603689e-32;
constexpr double kPio4 = 0.78539816339744828;   // the double below pi/4

// sin(r), cos(r) for a double-double |r| <= ~pi/4 + 2^-30: Taylor series in z = r^2.
// Terms k >= 9 of sin (k >= 10 of cos) contribute < 2^-60 relative and are summed in double.
PPCR_FN void sincos_kernel(dd r, dd& s, dd& c) {
    const dd z = mul(r, r);
    double ps = kSinH[12];
#pragma unroll
    for (int k = 11; k >= 8; k--) ps = fma_(ps, z.h, kSinH[k]);
    dd p = {ps, 0.0};
#pragma unroll
    for (int k = 7; k >= 0; k--) p = add(mul(p, z), dd{kSinH[k], kSinL[k]});
    s = add(r, mul(mul(r, z), p));
    double pc = kCosH[13];
#pragma unroll
    for (int k = 12; k >= 9; k--) pc = fma_(pc, z.h, kCosH[k]);
    dd q = {pc, 0.0};
#pragma unroll
    for (int k = 8; k >= 0; k--) q = add(mul(q, z), dd{kCosH[k], kCosL[k]});
    c = add(dd{1.0, 0.0}, mul(z, q));
}

// sin(x), cos(x) in double-double for |x| < kCrMax (finite). Returns false outside that range.
PPCR_FN bool sincos_dd(double x, dd& s, dd& c) {
    const bool negx = (bits(x) >> 63) != 0;
    const double ax = negx ? -x : x;
    if (!(ax < kCrMax)) return false;
    int n = 0;
    dd r = {ax, 0.0};
    if (ax > kPio4) {
        n = (int)(ax * 0.63661977236758138 + 0.5);
        const double fn = (double)n;
        const double r1 = ax - fn * kP1;                 // exact: fn * kP1 exact, Sterbenz
        r = two_sum(r1, -(fn * kP2));                     // fn * kP2 exact
        r = add(r, dd{-(fn * kP3), 0.0});                 // fn * kP3 exact
        r = add(r, neg(two_prod(fn, kP4)));
    }
    dd ks, kc;
    sincos_kernel(r, ks, kc);
    switch (n & 3) {
        case 0: s = ks; c = kc; break;
        case 1: s = kc; c = neg(ks); break;
        case 2: s = neg(ks); c = neg(kc); break;
        default: s = neg(kc); c = ks; break;
    }
    if (negx) s = neg(s);
    return true;
}

// correctly rounded sin(x) and cos(x) (|x| < kCrMax; false otherwise, outputs untouched)
PPCR_FN bool sincos(double x, double& s, double& c) {
    dd S, C;
    if (!sincos_dd(x, S, C)) return false;
    s = S.h + S.l;
    c = C.h + C.l;
    return true;
}

// atan2 correction of t0 (within a few ulp of atan2(y, x); finite nonzero y, x) and the sin/cos
// of the corrected angle. S0/C0 = sin/cos(t0) in double-double.
PPCR_FN double atan2_refine(double y, double x, double t0, dd S0, dd C0, double& s, double& c) {
    // scale (y, x) to moderate magnitudes: exact, atan2 is scale invariant
    const double m = (y < 0 ? -y : y) > (x < 0 ? -x : x) ? (y < 0 ? -y : y) : (x < 0 ? -x : x);
    const int e = (int)((bits(m) >> 52) & 0x7ff) - 1023;
    if (e > 400 || e < -400) {
        uint64_t u = (uint64_t)(1023 - e) << 52;      // 2^-e, a normal double for |e| <= 1022
        double sc;
        memcpy(&sc, &u, 8);
        y *= sc;
        x *= sc;
    }
    // num = y cos t0 - x sin t0 (cancels to ~|v| 2^-53: the leading products are exact-subtracted)
    const dd a = two_prod(y, C0.h), b = two_prod(x, S0.h);
    const double num = (a.h - b.h) + ((a.l - b.l) + (y * C0.l - x * S0.l));
    const double den = x * C0.h + y * S0.h;
    const double delta = num / den;                    // atan(delta) = delta (|delta| ~ 2^-52 t0)
    const double t = t0 + delta;
    const double eps = t - t0;                         // exact (t and t0 are neighbours or equal)
    // sin/cos(t0 + eps) = S0 + eps C0 - eps^2/2 S0, cos: C0 - eps S0 - eps^2/2 C0
    dd st = add(S0, add(two_prod(eps, C0.h), dd{eps * C0.l - 0.5 * eps * eps * S0.h, 0.0}));
    dd ct = add(C0, add(neg(two_prod(eps, S0.h)), dd{-eps * S0.l - 0.5 * eps * eps * C0.h, 0.0}));
    s = st.h + st.l;
    c = ct.h + ct.l;
    return t;
}

}  // namespace ppcr

// pp_numfmt.h — exact decimal <-> binary64 conversions for the wire codec, host and device.
//
// The reference reads numbers with strtod (json.hpp:2645) and writes them with "%.15g"
// (json.hpp:6694); both are correctly rounded (glibc: round-half-even on the exact value). These
// integer-only algorithms give the identical bits/text on their domains and report `false`
// outside them (the caller then falls back to libc on the host, or flags the message for the
// host on the device):
//   dec_to_double: value = M * 10^e10 with M < 2^64 (<= 19 significant digits), |e10| <= 27:
//     e10 >= 0: the integer M * 5^e10 < 2^127, rounded to 53 bits, times 2^e10;
//     e10 <  0: q = (M << s) / 5^k with >= 55 quotient bits and a sticky remainder, rounded to 53
//               bits, times 2^(-s-k). One rounding from the exact value in both cases.
//   fmt15g: 1e-13 <= |x| < 1e18: D = round-half-even(|x| * 10^(14 - E)) computed exactly in
//     128-bit integers (x = m * 2^q), E = floor(log10 |x|) (fixed up from an estimate), then the
//     %g layout (fixed for -4 <= X < 15, else d.ddde+XX; trailing zeros removed).
#pragma once
#include <stdint.h>
#include <string.h>

#ifndef PP_HD
#define PP_HD __host__ __device__
#endif

namespace ppnum {

typedef unsigned __int128 u128;

PP_HD inline uint64_t pow5(int k) {          // 5^k, k <= 27 (5^27 < 2^63)
    uint64_t r = 1;
    for (int i = 0; i < k; i++) r *= 5;
    return r;
}
PP_HD inline uint64_t pow10u(int k) {        // 10^k, k <= 19
    uint64_t r = 1;
    for (int i = 0; i < k; i++) r *= 10;
    return r;
}
PP_HD inline int bitlen64(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }
PP_HD inline int bitlen128(u128 x) {
    const uint64_t hi = (uint64_t)(x >> 64);
    return hi ? 64 + bitlen64(hi) : bitlen64((uint64_t)x);
}

// nearest double to (v + sticky fraction) * 2^e2, ties to even; v > 0; when sticky, v has >= 55 bits
PP_HD inline double round_u128(u128 v, int e2, bool sticky) {
    const int nb = bitlen128(v);
    if (nb <= 53) return ldexp((double)(uint64_t)v, e2);
    const int sh = nb - 53;
    uint64_t mant = (uint64_t)(v >> sh);
    const u128 rem = v & (((u128)1 << sh) - 1);
    const u128 half = (u128)1 << (sh - 1);
    int ex = e2 + sh;
    if (rem > half || (rem == half && (sticky || (mant & 1)))) {
        mant++;
        if (mant == (1ull << 53)) { mant >>= 1; ex++; }
    }
    return ldexp((double)mant, ex);
}

PP_HD inline bool dec_to_double(uint64_t M, int e10, bool neg, double* out) {
    if (M == 0) { *out = neg ? -0.0 : 0.0; return true; }
    if (e10 > 27 || e10 < -27) return false;
    double r;
    if (e10 >= 0) {
        r = round_u128((u128)M * pow5(e10), e10, false);
    } else {
        const int k = -e10;
        const uint64_t D = pow5(k);
        int s = 55 + bitlen64(D) - bitlen64(M);
        if (s < 0) s = 0;
        const u128 N = (u128)M << s;
        const u128 q = N / D;
        const u128 rm = N - q * D;
        r = round_u128(q, -s - k, rm != 0);
    }
    *out = neg ? -r : r;
    return true;
}

// Scans a JSON number at p (< e) into (M, e10): returns chars consumed (0: not a number), sets
// *fast = false when it has more than 19 significant digits or an exponent beyond +-99999.
// is_int: no fraction and no exponent (nlohmann's integer tokens).
PP_HD inline int scan_number(const char* p, const char* e, uint64_t* M, int* e10, bool* neg, bool* is_int,
                             bool* fast) {
    const char* s = p;
    *neg = false; *is_int = true; *fast = true;
    uint64_t m = 0;
    int nd = 0, ex = 0;
    bool lead = true;
    if (p < e && *p == '-') { *neg = true; p++; }
    if (p >= e || *p < '0' || *p > '9') return 0;
    if (*p == '0') {
        p++;
    } else {
        while (p < e && *p >= '0' && *p <= '9') {
            lead = false;
            if (nd < 19) { m = m * 10 + (uint64_t)(*p - '0'); nd++; }
            else { *fast = false; ex++; }
            p++;
        }
    }
    if (p < e && *p == '.') {
        p++;
        *is_int = false;
        if (p >= e || *p < '0' || *p > '9') return 0;
        while (p < e && *p >= '0' && *p <= '9') {
            if (lead && *p == '0') { ex--; p++; continue; }
            lead = false;
            if (nd < 19) { m = m * 10 + (uint64_t)(*p - '0'); nd++; ex--; }
            else *fast = false;
            p++;
        }
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
        p++;
        *is_int = false;
        bool en = false;
        if (p < e && (*p == '+' || *p == '-')) { en = *p == '-'; p++; }
        if (p >= e || *p < '0' || *p > '9') return 0;
        int v = 0;
        while (p < e && *p >= '0' && *p <= '9') {
            if (v < 100000) v = v * 10 + (*p - '0');
            else *fast = false;
            p++;
        }
        ex += en ? -v : v;
    }
    *M = m;
    *e10 = ex;
    return (int)(p - s);
}

// F = floor(|x| * 10^k) and up = round-half-even increment: x = m * 2^q
PP_HD inline bool scaled_floor(uint64_t m, int q, int k, uint64_t* F, bool* up) {
    if (k < 0) {
        // |x| / 10^j = (m * 2^q) / 10^j, or m / (10^j * 2^-q): |x| < 1e18 keeps both below 2^64
        const int j = -k;
        if (q > 10 || q < -52 || j > 17) return false;
        const u128 N = q >= 0 ? (u128)m << q : (u128)m;
        const u128 P = q >= 0 ? (u128)pow10u(j) : (u128)pow10u(j) << (-q);
        const u128 f = N / P, r = N - f * P;
        *F = (uint64_t)f;
        *up = 2 * r > P || (2 * r == P && (f & 1));
        return true;
    }
    if (k > 27) return false;
    const u128 v = (u128)m * pow5(k);
    const int e2 = q + k;
    if (e2 >= 0) {
        if (bitlen128(v) + e2 > 64) return false;
        *F = (uint64_t)(v << e2);
        *up = false;
        return true;
    }
    const int sh = -e2;
    if (sh >= 127) { *F = 0; *up = false; return true; }
    const u128 f = v >> sh, r = v & (((u128)1 << sh) - 1), half = (u128)1 << (sh - 1);
    if ((f >> 64) != 0) return false;
    *F = (uint64_t)f;
    *up = r > half || (r == half && (f & 1));
    return true;
}

// "%.15g" of a finite nonzero x into out (>= 32 bytes); returns length, 0 when outside the domain
PP_HD inline int fmt15g(double x, char* out) {
    if (!(x == x) || x == 0.0) return 0;
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    if (!(ax >= 1e-13 && ax < 1e18)) return 0;
    uint64_t bits;
    memcpy(&bits, &ax, 8);
    const int be = (int)((bits >> 52) & 0x7FF);
    const uint64_t m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    const int q = be - 1075;
    // E estimate from the binary exponent: log10(2) ~ 0.30103; then fix up
    int E = (int)((double)(be - 1023) * 0.30102999566398120);
    if (be - 1023 < 0) E -= 1;
    const uint64_t lo = 100000000000000ull, hi = 1000000000000000ull;   // 1e14, 1e15
    uint64_t D = 0;
    int X = 0;
    bool done = false;
    for (int it = 0; it < 4 && !done; it++) {
        uint64_t F;
        bool up;
        if (!scaled_floor(m, q, 14 - E, &F, &up)) return 0;
        if (F >= hi) { E++; continue; }
        if (F < lo) { E--; continue; }
        D = F + (up ? 1 : 0);
        X = E;
        if (D == hi) { D = lo; X = E + 1; }            // rounding carry: 1.00..0 * 10^(E + 1)
        done = true;
    }
    if (!done) return 0;
    if (D < lo || D >= hi) return 0;
    char dg[16];
    for (int i = 14; i >= 0; i--) { dg[i] = (char)('0' + D % 10); D /= 10; }
    int nd = 15;
    while (nd > 1 && dg[nd - 1] == '0') nd--;            // %g strips trailing zeros
    int n = 0;
    if (neg) out[n++] = '-';
    if (X < -4 || X >= 15) {
        out[n++] = dg[0];
        if (nd > 1) { out[n++] = '.'; for (int i = 1; i < nd; i++) out[n++] = dg[i]; }
        out[n++] = 'e';
        int ex = X;
        out[n++] = ex < 0 ? '-' : '+';
        if (ex < 0) ex = -ex;
        if (ex >= 100) { out[n++] = (char)('0' + ex / 100); ex %= 100; out[n++] = (char)('0' + ex / 10); out[n++] = (char)('0' + ex % 10); }
        else { out[n++] = (char)('0' + ex / 10); out[n++] = (char)('0' + ex % 10); }
    } else if (X >= 0) {
        for (int i = 0; i <= X; i++) out[n++] = i < nd ? dg[i] : '0';
        if (nd > X + 1) { out[n++] = '.'; for (int i = X + 1; i < nd; i++) out[n++] = dg[i]; }
    } else {
        out[n++] = '0';
        out[n++] = '.';
        for (int i = 0; i < -X - 1; i++) out[n++] = '0';
        for (int i = 0; i < nd; i++) out[n++] = dg[i];
    }
    return n;
}

}  // namespace ppnum

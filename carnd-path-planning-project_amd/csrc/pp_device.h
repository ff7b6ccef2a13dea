// pp_device.h — device-side planner stages (gfx950, FP64 VALU).
//
// Each function restates one reference routine (file:line of Fable3/CarND-Path-Planning-Project)
// in the reference's floating-point evaluation order; the library is built with -ffp-contract=off
// so no mul+add pair is fused. Only transcendentals (atan2/sin/cos from the ROCm device math
// library) can differ from glibc by an ulp: parity is within 1e-6 m (measured ~1e-12 m).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pp.h"
#include "pp_math.h"

#ifndef PP_DIAGC   // branch-event census hook (pp_eval.hip, PP_DIAG builds)
#define PP_DIAGC(k, c) ((void)0)
#endif

#ifndef PP_WGRID
#define PP_WGRID 1          // the closest-waypoint cell table (init_reference_waypoint); 0: A/B builds
#endif
#ifndef PP_KDIV
#define PP_KDIV 1           // K1's table reciprocals (project_speed, lane matching's last quotient)
#endif

namespace ppd {

constexpr double kPi = 3.14159265358979323846;   // helpers.h:33
constexpr double kEps = 1e-5;                     // src/main.cpp:24
constexpr int kKP = 17;                       // LDS knot stride (16 knots + 1 pad: bank spread)
static_assert(kKP >= 15, "a slot holds npk + ncp <= (PP_PREV_KEEP - 1) + 6 = 15 knots");
constexpr int NL = PP_NUM_LANES;                  // lanes (src/main.cpp:22)
// ref x/y, normal x/y, lane centre x[NL]/y[NL], length[NL], segment |.|^2 [NL] and its reciprocal [NL]
constexpr int kMapArrays = 4 + 5 * NL;

// Map geometry (SoA). Arrays [i] or [lane * n + i]. llen[lane*n+i] = |lc[i] - lc[i-1]|
// (Map::get_lane_length, src/main.cpp:138-142), precomputed on the host with the same formula.
// lden[lane*n+i] = (ax - bx)^2 + (ay - by)^2 for a = lc[i-1], b = lc[i]: distancesq_pt_seg's rdenom
// (helpers.h:202) for that lane segment, and lrcp = RN(1 / lden). fastm: every lden lies in
// [2^-500, 2^500] (no degenerate lane segment), so lane_matching may use the tables.
// The closest-waypoint cell table (host build_wgrid): for a square cell of side 1 / ginv near the
// road, the (at most 4) waypoints that can be the closest one to any point of the cell, ascending,
// the last repeated; 0xFFFFFFFF in .x: no list (the full scan). Cell (i, j) at wgrid[j * gnx + i]
// covers [gx0 + i / ginv, gx0 + (i + 1) / ginv) x [gy0 + j / ginv, ...).
struct WGrid {
    const uint2* cells = nullptr;
    double gx0 = 0, gy0 = 0, ginv = 0;
    int gnx = 0, gny = 0;
};
struct MapV {
    const double *ref_x, *ref_y, *nx, *ny, *lc_x, *lc_y, *llen, *lden, *lrcp;
    int n;
    int fastm;
    WGrid wg;
    // reference segments (build_wseg): wseg[b] = (|ref_b - ref_{b-1}|, RN(1 / that)), the length
    // Map::project_speed computes (src/main.cpp:339) and its correctly rounded reciprocal; null:
    // computed in place
    const double2* wseg = nullptr;
    // the approach table (pp_eval.hip build_atab): kAtabD doubles per lane segment b, used where
    // atab_on (k_prep: in LDS when the map is, so that its loads are LDS loads)
    const double* atab = nullptr;
    bool atab_on = false;
};
// approach table row b (the lane segments from waypoint b - 1 to b): dx_l, dy_l at 2 l, 2 l + 1 (the
// walk's own RN(pb - pa)), kf_l at 2 NL + l, kb_l at 3 NL + l, the segment length llen_l at 4 NL + l
// (l < NL)
constexpr int kAtabD = (5 * NL + 1) & ~1;
// margin of the certain approach test, m^2 (approach_cert)
constexpr double kAtabMargin = 1e-3;

// Per-scene preparation output of K1 (SoA, workspace).
struct PrepV {
    double *pos_x, *pos_y, *angle, *ca_m, *sa_m, *ca_p, *sa_p;
    double *ego_speed, *ego_d, *ego_vd, *ratio /*[NL][S]*/, *in_ts, *in_tt, *l_ts /*[NL][S]*/,
        *l_tt /*[NL][S]*/, *score /*[NL][S]*/;
    int32_t *K, *ref_wp, *T, *ego_lane, *open_mask, *lim_mask, *status;
};

// src/main.cpp:134-137 (idx + size) % size, size_t arithmetic
__device__ __attribute__((noinline)) int wpi_far(int idx, int n) {
    if (idx >= 0) return idx % n;
    return (int)(((uint64_t)(int64_t)idx + (uint64_t)n) % (uint64_t)n);
}
// Every index the walks form lies within one map length of [0, n) (a walk steps one waypoint at a
// time from a valid index; the prefetches look a few waypoints ahead), where the wrap is one
// compare and one add or subtract. Further out (tiny maps, walks round the loop) the integer
// remainder, out of line: inline, the compiler evaluated its ~12-instruction sequence for every
// index and selected the result (PP_WPI_FAST=0 keeps that form)
#ifndef PP_WPI_FAST
#define PP_WPI_FAST 1
#endif
__device__ __forceinline__ int wpi(int idx, int n) {
    if (!PP_WPI_FAST) {
        if (idx >= 0) return idx < n ? idx : idx % n;
        if (idx >= -n) return idx + n;
        return (int)(((uint64_t)(int64_t)idx + (uint64_t)n) % (uint64_t)n);
    }
    const int hi = idx - n, lo = idx + n;
    if (__builtin_expect(idx >= -n && hi < n, 1)) return idx < 0 ? lo : (idx < n ? idx : hi);
    return wpi_far(idx, n);
}
__device__ __forceinline__ double lane_offset(int lane) { return 4.0 * (lane + 0.5); }  // :84-88
__device__ __forceinline__ double s_min(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ double s_max(double a, double b) { return (a < b) ? b : a; }  // std::max

// helpers.h:188-249 distancesq_pt_seg
__device__ __forceinline__ double distsq_pt_seg(double px, double py, double ax, double ay, double bx,
                                                double by, double& rnom_o, double& rdenom_o,
                                                double& snom_o) {
    rnom_o = 0; rdenom_o = 1; snom_o = 0;
    if (ax == bx && ay == by) return (ax - bx) * (ax - bx) + (ay - by) * (ay - by);
    const double rdenom = (ax - bx) * (ax - bx) + (ay - by) * (ay - by);
    const double pdx = px - ax, dx = bx - ax;
    const double pdy = py - ay, dy = by - ay;
    const double rnom = pdx * dx + pdy * dy;
    rdenom_o = rdenom;
    const double snom = pdx * dy - pdy * dx;
    snom_o = snom;
    if (rnom < -1) { rnom_o = 0; return (px - ax) * (px - ax) + (py - ay) * (py - ay); }
    if (rnom > rdenom) { rnom_o = rdenom; return (px - bx) * (px - bx) + (py - by) * (py - by); }
    rnom_o = rnom;
    return snom * snom / rdenom;
}

// Map::init_reference_waypoint (src/main.cpp:143-197) from the closest waypoint on (:150-154 done
// by the caller)
__device__ inline void init_reference_waypoint_from(const MapV& m, double x, double y, int closest,
                                                    int& ref_wp, double ratio[NL]) {
    const int n = m.n;
    double rnom, snom, rdenom, d0, d1;
    {
        const int a = wpi(closest - 1, n), b = wpi(closest, n), c = wpi(closest + 1, n);
        d0 = distsq_pt_seg(x, y, m.ref_x[a], m.ref_y[a], m.ref_x[b], m.ref_y[b], rnom, rdenom, snom);
        d1 = distsq_pt_seg(x, y, m.ref_x[b], m.ref_y[b], m.ref_x[c], m.ref_y[c], rnom, rdenom, snom);
        if (d1 < d0) {
            closest++;
        } else if (d1 == d0) {
            const double anx = (m.nx[a] + m.nx[b]) / 2, any = (m.ny[a] + m.ny[b]) / 2;
            const double dpx = x - m.ref_x[b], dpy = y - m.ref_y[b];
            const double dotp = anx * dpx + any * dpy;
            if (dotp > 0) closest++;
        }
    }
    ref_wp = closest;
    const int a = wpi(closest - 1, n), b = wpi(closest, n);
    for (int lane = 0; lane < NL; lane++) {
        distsq_pt_seg(x, y, m.lc_x[lane * n + a], m.lc_y[lane * n + a], m.lc_x[lane * n + b],
                      m.lc_y[lane * n + b], rnom, rdenom, snom);
        ratio[lane] = rnom / rdenom;
    }
}

// Map::init_reference_waypoint (src/main.cpp:143-197)
__device__ inline void init_reference_waypoint(const MapV& m, double x, double y, int& ref_wp,
                                               double ratio[NL]) {
    const int n = m.n;
    int closest = 0;
    // the closest waypoint (:150-154): the first i with the smallest |ref_i - p|^2 (strict `d < cd`
    // from d_0). Near the road the cell table holds every waypoint that can be it for a point of the
    // cell (ascending): the same scan over them gives the same index, since the first minimal index
    // of the whole map is among them and no smaller listed index reaches the minimum (build_wgrid);
    // elsewhere (and for NaN or infinite positions) the full scan
    bool scan = true;
    if (PP_WGRID && m.wg.cells) {
        const double fx = (x - m.wg.gx0) * m.wg.ginv, fy = (y - m.wg.gy0) * m.wg.ginv;
        if (fx >= 0 && fy >= 0 && fx < (double)m.wg.gnx && fy < (double)m.wg.gny) {
            const uint2 c = m.wg.cells[(int64_t)(int)fy * m.wg.gnx + (int)fx];
            if (c.x != 0xFFFFFFFFu) {
                scan = false;
                const int i0 = (int)(c.x & 0xFFFFu), i1 = (int)(c.x >> 16), i2 = (int)(c.y & 0xFFFFu),
                          i3 = (int)(c.y >> 16);
                double cd;
                { const double dx = m.ref_x[i0] - x, dy = m.ref_y[i0] - y; cd = dx * dx + dy * dy; }
                closest = i0;
                const int ix[3] = {i1, i2, i3};
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const double dx = m.ref_x[ix[k]] - x, dy = m.ref_y[ix[k]] - y;
                    const double d = dx * dx + dy * dy;
                    if (d < cd) { closest = ix[k]; cd = d; }
                }
            }
        }
    }
    if (scan) {
        double cd;
        { const double dx = m.ref_x[0] - x, dy = m.ref_y[0] - y; cd = dx * dx + dy * dy; }
        for (int i = 1; i < n; i++) {
            const double dx = m.ref_x[i] - x, dy = m.ref_y[i] - y;
            const double d = dx * dx + dy * dy;
            if (d < cd) { closest = i; cd = d; }
        }
    }
    init_reference_waypoint_from(m, x, y, closest, ref_wp, ratio);
}

// The same, the closest-waypoint scan (:150-154: the first i with the smallest |ref_i - p|^2 under
// `d < cd` from cd = d_0) split over the G lanes of a group (lane r scans i = r, r + G, ...) and
// reduced by (distance, index). Equal to the serial scan: a NaN d_i never wins `d < cd`, a NaN d_0
// keeps waypoint 0, and no finite-or-infinite d below d_0 keeps waypoint 0 as well.
template <int G>
__device__ inline void init_reference_waypoint_grp(const MapV& m, double x, double y, int r,
                                                   int& ref_wp, double ratio[NL]) {
    const int n = m.n;
    int closest = -1;
    double cd = __builtin_inf();
    for (int i = r; i < n; i += G) {
        const double dx = m.ref_x[i] - x, dy = m.ref_y[i] - y;
        const double d = dx * dx + dy * dy;
        if (d < cd) { closest = i; cd = d; }
    }
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
        const double od = __shfl_xor(cd, o, G);
        const int oc = __shfl_xor(closest, o, G);
        if (oc >= 0 && (closest < 0 || od < cd || (od == cd && oc < closest))) { cd = od; closest = oc; }
    }
    const double dx0 = m.ref_x[0] - x, dy0 = m.ref_y[0] - y;
    const double d0 = dx0 * dx0 + dy0 * dy0;
    if (closest < 0 || !(d0 == d0) || !(cd < d0)) closest = 0;
    init_reference_waypoint_from(m, x, y, closest, ref_wp, ratio);
}

// Map::lane_matching (src/main.cpp:199-275); bounded walk (never reached on finite input).
// The reference computes s, d, lane and next_wp at every improvement (:214-227); only the last
// improvement's values survive, so the walk records that projection's raw terms (lane, segment,
// rnom, rdenom, snom, the lane's running sum_s and ratio shift) and evaluates the same
// expressions once after the walk: identical results, one division and one sqrt per walk.
__device__ inline bool lane_matching(const MapV& m, int ref_wp, const double ratio[NL], double x,
                                     double y, double& out_s, double& out_d, int& out_lane,
                                     int& out_next_wp) {
    const int n = m.n;
    int dir = 0;
    bool stop = false;
    int cur = ref_wp;
    double sum_s[NL], sr[NL];
#pragma unroll
    for (int l = 0; l < NL; l++) { sum_s[l] = 0; sr[l] = ratio[l]; }
    double best = 1000 * 1000;
    bool found = false;
    int b_lane = 0, b_cur = 0;
    double b_rnom = 0, b_rdenom = 1, b_snom = 0, b_ss = 0, b_sr = 0;
    for (int it = 0; it < 4 * n + 8; it++) {
        PP_DIAGC(16, true);
        bool improved = false;
        const int a = wpi(cur - 1, n), b = wpi(cur, n);
#pragma unroll
        for (int lane = 0; lane < NL; lane++) {
            double rnom, snom, rdenom;
            const double dsq = distsq_pt_seg(x, y, m.lc_x[lane * n + a], m.lc_y[lane * n + a],
                                             m.lc_x[lane * n + b], m.lc_y[lane * n + b], rnom,
                                             rdenom, snom);
            if (dsq < best) {
                best = dsq;
                improved = true;
                found = true;
                b_lane = lane;
                b_cur = cur;
                b_rnom = rnom; b_rdenom = rdenom; b_snom = snom;
                b_sr = sr[lane];
                b_ss = sum_s[lane];
            }
            if (rnom == 0) {
                if (dir == 1) stop = true;
                dir = -1;
            } else if (rnom == rdenom) {
                if (dir == -1) stop = true;
                dir = 1;
            } else {
                stop = true;
            }
        }
        if (!improved || stop) break;
        double ll[NL];
#pragma unroll
        for (int l = 0; l < NL; l++) ll[l] = m.llen[l * n + b];
        if (dir > 0) {
#pragma unroll
            for (int l = 0; l < NL; l++) { sum_s[l] += (1 - sr[l]) * ll[l]; sr[l] = 0; }
            cur++;
        } else {
#pragma unroll
            for (int l = 0; l < NL; l++) { sum_s[l] -= sr[l] * ll[l]; sr[l] = 1; }
            cur--;
        }
    }
    if (found) {                                                   // :214-227, last improvement
        const double rfs = b_rnom / b_rdenom;
        const double r_mod = rfs - b_sr;
        const double seg_len = m.llen[b_lane * n + wpi(b_cur, n)];
        out_s = b_ss + seg_len * r_mod;
        double d = sqrt(best);
        if (b_snom < 0) d = -d;
        out_d = d + lane_offset(b_lane);
        out_lane = b_lane;
        out_next_wp = b_cur;
    }
    return found;
}

// n / d correctly rounded from r = RN(1/d) (Markstein: q0 = RN(n r) is within an ulp of n/d, the
// residual n - q0 d is exact by fma, and RN(q0 + residual r) is RN(n/d)), for d in [2^-500, 2^500]
// and n = 0 or |n| in [2^-400, 2^400] (the quotient stays normal; 4e8 random operands in these
// ranges, many with near-all-ones divisor significands, agree with IEEE division bit for bit);
// elsewhere the IEEE division.
__device__ __forceinline__ double div_by_rcp(double n, double d, double r) {
    const double q0 = n * r;
    const double q = __builtin_fma(__builtin_fma(-q0, d, n), r, q0);
    const double an = fabs(n);
    if (__builtin_expect(!((an >= 0x1p-400 && an <= 0x1p400) || an == 0.0), 0)) return n / d;
    return an == 0.0 ? q0 : q;
}

// One walk iteration's segment (a, b) is an *approach* segment when every lane's projection is
// clamped to the end the walk moves towards (rn > rdenom forward, rn < -1 backward: the walk goes
// on in the same direction, src/main.cpp:237-246), on a map whose lane segments all have rdenom >=
// 1 m^2 and lane centres within 4e4 m of the origin (MapV::fastm bit 2, checked once per map) for a
// point within 5e4 m of it (so within 1e5 m of every lane point; checked once per walk): then every lane's squared distance at this iteration is below its value at the previous one
// by more than rdenom minus the rounding of rn (exact: |p-a|^2 - |p-b|^2 = 2 (rn - rdenom) + rdenom),
// far more than the rounding of the distances themselves (< 1e-5 m^2 there), so the iteration
// improves the running minimum whatever it was. rn is computed by the walk's own operations.
__device__ __forceinline__ bool approach_seg(const MapV& m, int a, int b, double x, double y, bool fwd) {
    const int n = m.n;
    bool okf = true, okb = true;          // every lane's test, no short circuit (no branches)
#pragma unroll
    for (int lane = 0; lane < NL; lane++) {
        const double pax = m.lc_x[lane * n + a], pay = m.lc_y[lane * n + a];
        const double pbx = m.lc_x[lane * n + b], pby = m.lc_y[lane * n + b];
        const double den = m.lden[lane * n + b];
        const double pdx = x - pax, dx = pbx - pax;
        const double pdy = y - pay, dy = pby - pay;
        const double rn = pdx * dx + pdy * dy;
        okf &= rn > den;
        okb &= rn < -1;
    }
    return fwd ? okf : okb;
}
// A *certain* approach segment (MapV::atab; maps with fastm bit 2, a point within 5e4 m of the
// origin): per lane, t = x dx + y dy - k by two fmas, k = pa.d + rdenom + kAtabMargin (forward) or
// pa.d - 1 - kAtabMargin (backward), d = (dx, dy). In real arithmetic t is the walk's rn - rdenom -
// kAtabMargin (forward; rn + 1 + kAtabMargin backward) up to the roundings of k and of the two fmas;
// under the fastm bounds (|x|, |y| < 5e4, lane centres within 4e4, |d| < 8e4) those and the walk's
// own rounding of rn stay below 2e-5 m^2, far inside the margin: t > 0 (t < 0 backward) implies the
// walk's rn > rdenom (rn < -1) for every lane, i.e. approach_seg. A segment it does not certify is
// left to the full walk (approach runs stop there), which is always exact.
__device__ __forceinline__ bool approach_cert(const MapV& m, int b, double x, double y, bool fwd) {
    const double* r = m.atab + b * kAtabD;
    const double* kr = r + (fwd ? 2 * NL : 3 * NL);
    double d[2 * NL], k[NL];
#pragma unroll
    for (int l = 0; l < 2 * NL; l++) d[l] = r[l];
#pragma unroll
    for (int l = 0; l < NL; l++) k[l] = kr[l];
    const double sg = fwd ? 1.0 : -1.0;     // (t sg > 0: exact, and false for t = 0 either way)
    bool ok = true;
#pragma unroll
    for (int l = 0; l < NL; l++) ok &= __builtin_fma(x, d[2 * l], __builtin_fma(y, d[2 * l + 1], -k[l])) * sg > 0;
    return ok;
}
#ifndef PP_ATAB
#define PP_ATAB 1
#endif
__device__ __forceinline__ bool approach_test(const MapV& m, int a, int b, double x, double y, bool fwd) {
    return (PP_ATAB && m.atab_on) ? approach_cert(m, b, x, y, fwd) : approach_seg(m, a, b, x, y, fwd);
}
// commits approach segments from iteration `it` (segment (a, b), an approach segment) while the
// next one is one too; returns the iteration the full walk resumes at (its segment uncommitted).
// After the walk's first step the ratio shift sr is 0 forward and 1 backward, so a commit adds or
// subtracts the segment length exactly ((1 - 0) l = l, 1 l = l; x - l == x + (-l)).
__device__ __forceinline__ int approach_walk(const MapV& m, double x, double y, int dir, int& a, int& b,
                                             int& cur, double sum_s[NL], int it) {
    const int n = m.n;
    const bool fwd = dir > 0;
    for (;;) {
        if (it + 2 >= 4 * n + 8 || cur - 2 < -n) break;
        const int a2 = fwd ? b : (a == 0 ? n - 1 : a - 1);
        const int b2 = fwd ? (b + 1 == n ? 0 : b + 1) : a;
        // the committed segment's lengths, read before the test (with the table: from its row, in
        // the same round trip to LDS as the tested row)
        double len[NL];
#pragma unroll
        for (int l = 0; l < NL; l++)
            len[l] = (PP_ATAB && m.atab_on) ? m.atab[b * kAtabD + 4 * NL + l] : m.llen[l * n + b];
        if (!approach_test(m, a2, b2, x, y, fwd)) break;
        PP_DIAGC(24, true);
#pragma unroll
        for (int l = 0; l < NL; l++) sum_s[l] += fwd ? len[l] : -len[l];
        cur += dir;
        a = a2; b = b2;
        it++;
    }
    return it;
}

// lane_matching on a map with fastm: the same walk, with each lane segment's rdenom and its
// reciprocal from the tables (the division snom^2 / rdenom by div_by_rcp: the same correctly
// rounded value), the waypoint indices stepped instead of re-wrapped, and lighter bookkeeping
// (same arithmetic, same results):
// - the walk is monotone (a direction change stops it, :237-246), so a segment's end points are
//   carried to the next iteration (forward: b becomes a; backward: a becomes b) and only the new
//   point is loaded;
// - an improvement records only its lane (and the best distance); the iteration's segment, the
//   lane's running sum_s and ratio shift are kept once per improving iteration, and the recorded
//   projection's rnom/snom are recomputed after the walk by the same operations;
// - a run of approach segments (approach_seg) is walked by its clamp tests and the sum_s
//   bookkeeping alone: each improves and goes on (nothing recorded there is read, since the next
//   iteration improves too), so only the last one before a segment that is not an approach segment
//   runs in full — it improves against any running minimum at least the true one (the kept
//   first-iteration minimum), and records the lane of its own minimum, as the full walk does.
//   The run starts after the first iteration (which sets the direction and a minimum below the
//   initial 1000^2) and stops one segment early.
__device__ inline bool lane_matching_tab2(const MapV& m, int ref_wp, const double ratio[NL], double x,
                                          double y, double& out_s, double& out_d, int& out_lane,
                                          int& out_next_wp) {
    const int n = m.n;
    int dir = 0;
    bool stop = false;
    int cur = ref_wp;
    int a = wpi(cur - 1, n), b = wpi(cur, n);
    double sum_s[NL], sr[NL];
#pragma unroll
    for (int l = 0; l < NL; l++) { sum_s[l] = 0; sr[l] = ratio[l]; }
    double best = 1000 * 1000;
    bool found = false;
    int b_lane = 0, k_cur = 0, k_b = 0, k_a = 0;
    double k_ss = 0, k_sr = 0;
    for (int it = 0; it < 4 * n + 8; it++) {
        PP_DIAGC(16, true);
        bool improved = false;
        int il = 0;
#pragma unroll
        for (int lane = 0; lane < NL; lane++) {
            const double pax = m.lc_x[lane * n + a], pay = m.lc_y[lane * n + a];
            const double pbx = m.lc_x[lane * n + b], pby = m.lc_y[lane * n + b];
            const double den = m.lden[lane * n + b];
            const double pdx = x - pax, dx = pbx - pax;                        // helpers.h:203-207
            const double pdy = y - pay, dy = pby - pay;
            const double rn = pdx * dx + pdy * dy;
            double rnom, dsq;
            if (rn < -1) { rnom = 0; dsq = pdx * pdx + pdy * pdy; }                                       // :227-231
            else if (rn > den) { rnom = den; dsq = (x - pbx) * (x - pbx) + (y - pby) * (y - pby); }       // :232-236
            else {
                const double snom = pdx * dy - pdy * dx;
                rnom = rn; dsq = div_by_rcp(snom * snom, den, m.lrcp[lane * n + b]);
            }
            if (dsq < best) { best = dsq; improved = true; il = lane; }
            if (rnom == 0) {
                if (dir == 1) stop = true;
                dir = -1;
            } else if (rnom == den) {
                if (dir == -1) stop = true;
                dir = 1;
            } else {
                stop = true;
            }
        }
        if (improved) {          // this iteration holds the last improvement so far
            found = true;
            b_lane = il; k_cur = cur; k_a = a; k_b = b;
            k_ss = sum_s[0]; k_sr = sr[0];
#pragma unroll
            for (int l = 1; l < NL; l++) if (il == l) { k_ss = sum_s[l]; k_sr = sr[l]; }
        }
        if (!improved || stop) break;
        if (dir > 0) {
#pragma unroll
            for (int l = 0; l < NL; l++) { sum_s[l] += (1 - sr[l]) * m.llen[l * n + b]; sr[l] = 0; }
            cur++;
            a = b;
            b = b + 1 == n ? 0 : b + 1;
            if (__builtin_expect(cur - 1 < -n, 0)) { a = wpi(cur - 1, n); b = wpi(cur, n); }
        } else {
#pragma unroll
            for (int l = 0; l < NL; l++) { sum_s[l] -= sr[l] * m.llen[l * n + b]; sr[l] = 1; }
            cur--;
            b = a;
            a = a == 0 ? n - 1 : a - 1;
            if (__builtin_expect(cur - 1 < -n, 0)) { a = wpi(cur - 1, n); b = wpi(cur, n); }
        }
        if (it == 0 && (m.fastm & 2) && fabs(x) < 5e4 && fabs(y) < 5e4 &&
            approach_test(m, a, b, x, y, dir > 0))
            it = approach_walk(m, x, y, dir, a, b, cur, sum_s, it + 1) - 1;
    }
    if (found) {                                                   // :214-227, last improvement
        const int l = b_lane;
        const double pax = m.lc_x[l * n + k_a], pay = m.lc_y[l * n + k_a];
        const double pbx = m.lc_x[l * n + k_b], pby = m.lc_y[l * n + k_b];
        const double den = m.lden[l * n + k_b];
        const double pdx = x - pax, dx = pbx - pax;
        const double pdy = y - pay, dy = pby - pay;
        const double rn = pdx * dx + pdy * dy;
        const double snom = pdx * dy - pdy * dx;
        const double rnom = rn < -1 ? 0.0 : (rn > den ? den : rn);
        // rnom / den by the table's RN(1 / den) (div_by_rcp: the correctly rounded quotient)
        const double rfs = PP_KDIV ? div_by_rcp(rnom, den, m.lrcp[l * n + k_b]) : rnom / den;
        const double r_mod = rfs - k_sr;
        const double seg_len = m.llen[l * n + k_b];
        out_s = k_ss + seg_len * r_mod;
        double d = sqrt(best);
        if (snom < 0) d = -d;
        out_d = d + lane_offset(l);
        out_lane = l;
        out_next_wp = k_cur;
    }
    return found;
}

__device__ __forceinline__ bool lane_match(const MapV& m, int ref_wp, const double ratio[NL], double x,
                                           double y, double& out_s, double& out_d, int& out_lane,
                                           int& out_next_wp) {
    if (m.fastm) return lane_matching_tab2(m, ref_wp, ratio, x, y, out_s, out_d, out_lane, out_next_wp);
    return lane_matching(m, ref_wp, ratio, x, y, out_s, out_d, out_lane, out_next_wp);
}

// Map::project_speed (src/main.cpp:330-358)
__device__ inline void project_speed(const MapV& m, double vx, double vy, int next_wp, double& vs,
                                     double& vd) {
    const int n = m.n;
    const int a = wpi(next_wp - 1, n), b = wpi(next_wp, n);
    double wx = m.ref_x[b] - m.ref_x[a], wy = m.ref_y[b] - m.ref_y[a];
    double2 ws = {0, 0};
    if (PP_KDIV && m.wseg) ws = m.wseg[b];              // (loaded ahead of the sqrt below)
    const double svl = sqrt(vx * vx + vy * vy);
    if (svl < kEps) {
        vs = svl;
        vd = 0;
        return;
    }
    double q;
    if (PP_KDIV && m.wseg) {
        // wvl = sqrt(wx^2 + wy^2) is the table's (the host computes it with the same operations,
        // correctly rounded sqrt), svl / wvl by its RN(1 / wvl): the same bits
        q = div_by_rcp(svl, ws.x, ws.y);
    } else {
        const double wvl = sqrt(wx * wx + wy * wy);
        q = svl / wvl;
    }
    wx *= q;
    wy *= q;
    double sign = 1.0;
    if (wx * vx + wy * vy < 0) { vx *= -1; vy *= -1; sign = -1; }
    double rnom, rdenom, snom;
    distsq_pt_seg(vx, vy, 0.0, 0.0, wx, wy, rnom, rdenom, snom);
    vs = (rnom / rdenom) * svl * sign;
    vd = (snom / rdenom) * svl * sign;
}

// get_lane_pos for K increasing positive targets s[0..K) in one forward walk. Every call with
// s > 0 walks forward only (s stays > 0 until s <= remaining_length, :291-302), through the same
// segments with the same remaining lengths, so target i sees exactly its own call's sequence of
// subtractions and stops where that call stops: identical points and ok flags.
template <int K>
__device__ inline void get_lane_pos_multi(const MapV& m, int ref_wp, double ratio, const double* s_in, int lane,
                                          double* ox, double* oy, bool* ok) {
    const int n = m.n;
    double sv[K];
    unsigned pending = (1u << K) - 1;
#pragma unroll
    for (int i = 0; i < K; i++) { sv[i] = s_in[i]; ok[i] = false; ox[i] = 0; oy[i] = 0; }
    int wp = ref_wp;
    double nx_ = 0, ny_ = 0, px_ = 0, py_ = 0;
    for (int it = 0; it < 4 * n + 8 && pending; it++) {
        const int b = wpi(wp, n), a = wpi(wp - 1, n);
        nx_ = m.lc_x[lane * n + b]; ny_ = m.lc_y[lane * n + b];
        px_ = m.lc_x[lane * n + a]; py_ = m.lc_y[lane * n + a];
        const double wl = m.llen[lane * n + b];
        const double rem = wl * (1 - ratio);
#pragma unroll
        for (int i = 0; i < K; i++) {
            if (!((pending >> i) & 1)) continue;
            if (sv[i] <= rem) {
                const double dest = 1 - (rem - sv[i]) / wl;
                ox[i] = nx_ * dest + px_ * (1 - dest);
                oy[i] = ny_ * dest + py_ * (1 - dest);
                ok[i] = true;
                pending &= ~(1u << i);
            } else {
                sv[i] -= rem;
            }
        }
        ratio = 0;
        wp++;
    }
    // a target the bounded walk did not reach: its call ends on the last segment with dest 0
#pragma unroll
    for (int i = 0; i < K; i++)
        if ((pending >> i) & 1) { ox[i] = nx_ * 0.0 + px_ * (1 - 0.0); oy[i] = ny_ * 0.0 + py_ * (1 - 0.0); }
}

// Map::get_lane_pos for a target s > 0: the walk only moves forward (s stays > 0, :291-302). The
// first kPf segments' lane-centre points and lengths are loaded up front, so their global-memory
// latencies overlap instead of chaining one per step; same arithmetic, same result.
template <int kPf>
__device__ inline void get_lane_pos_fwd(const MapV& m, int ref_wp, double ratio, double s, int lane,
                                        double& ox, double& oy, bool& ok) {
    const int n = m.n;
    const double* cx = m.lc_x + lane * n;
    const double* cy = m.lc_y + lane * n;
    const double* cl = m.llen + lane * n;
    double qx[kPf + 1], qy[kPf + 1], ql[kPf + 1];
#pragma unroll
    for (int k = 0; k <= kPf; k++) {
        const int b = wpi(ref_wp - 1 + k, n);
        qx[k] = cx[b]; qy[k] = cy[b]; ql[k] = cl[b];
    }
    ok = false;
    double dest = 0, nx_ = 0, ny_ = 0, px_ = 0, py_ = 0;
#pragma unroll
    for (int k = 0; k < kPf; k++) {
        nx_ = qx[k + 1]; ny_ = qy[k + 1]; px_ = qx[k]; py_ = qy[k];
        const double wl = ql[k + 1];
        const double rem = wl * (1 - ratio);
        if (s <= rem) { dest = 1 - (rem - s) / wl; ok = true; break; }
        s -= rem;
        ratio = 0;
    }
    if (!ok) {
        int wp = ref_wp + kPf;
        for (int it = kPf; it < 4 * n + 8; it++) {
            const int b = wpi(wp, n), a = wpi(wp - 1, n);
            nx_ = cx[b]; ny_ = cy[b]; px_ = cx[a]; py_ = cy[a];
            const double wl = cl[b];
            const double rem = wl * (1 - ratio);
            if (s <= rem) { dest = 1 - (rem - s) / wl; ok = true; break; }
            s -= rem;
            ratio = 0;
            wp++;
        }
    }
    ox = nx_ * dest + px_ * (1 - dest);
    oy = ny_ * dest + py_ * (1 - dest);
}

// Map::get_lane_pos (src/main.cpp:277-328) on one lane. ok=false if the bounded walk ran out.
__device__ inline void get_lane_pos(const MapV& m, int ref_wp, double ratio, double s, int lane,
                                    double& ox, double& oy, bool& ok) {
    const int n = m.n;
    int wp = ref_wp;
    double nx_ = 0, ny_ = 0, px_ = 0, py_ = 0, dest = 0;
    ok = false;
    for (int it = 0; it < 4 * n + 8; it++) {
        const int b = wpi(wp, n), a = wpi(wp - 1, n);
        nx_ = m.lc_x[lane * n + b]; ny_ = m.lc_y[lane * n + b];
        px_ = m.lc_x[lane * n + a]; py_ = m.lc_y[lane * n + a];
        const double wl = m.llen[lane * n + b];
        if (s > 0) {
            const double rem = wl * (1 - ratio);
            if (s <= rem) { dest = 1 - (rem - s) / wl; ok = true; break; }
            s -= rem;
            ratio = 0;
            wp++;
        } else {
            const double rem = wl * ratio;
            if (-s <= rem) { dest = (rem + s) / wl; ok = true; break; }
            s += rem;
            ratio = 1;
            wp--;
        }
    }
    ox = nx_ * dest + px_ * (1 - dest);
    oy = ny_ * dest + py_ * (1 - dest);
}

// SpeedController (src/main.cpp:488-548)
struct SC { double start, target, ttime, shift; };
__device__ __forceinline__ double sc_get_speed(const SC& c, double t) {
    t -= c.shift;
    if (t < 0) t = 0;
    if (t > c.ttime) return c.target;
    return c.start + (c.target - c.start) * t / c.ttime;
}
// sc_get_speed with r ~ 1/ttime (ppm::div_rcp): the same quotient
// kChecked = false: ramp times known in range (k_prep's check; k_cand<false>), no range checks
template <bool kChecked = true>
__device__ __forceinline__ double sc_get_speed_r(const SC& c, double t, double r) {
    t -= c.shift;
    // unchecked: t - shift is never NaN (finite in-range operands), so max(t, 0) is v_max_f64
    if (kChecked) { if (t < 0) t = 0; } else t = __builtin_fmax(t, 0.0);
    if (t > c.ttime) return c.target;
    return c.start + (kChecked ? ppm::div_rcp((c.target - c.start) * t, c.ttime, r)
                               : ppm::div_rcp_nc((c.target - c.start) * t, c.ttime, r));
}
__device__ __forceinline__ void sc_add_limit(SC& c, double nts, double ntt) {
    const double tm = s_max(c.ttime, 0.02);
    const double ntm = s_max(ntt, 0.02);
    const double cg = (c.target - c.start) / tm;
    const double ng = (nts - c.start) / ntm;
    if (ng < cg) { c.target = nts; c.ttime = ntt; }
}
__device__ __forceinline__ void sc_override(SC& c, double t, double speed) {
    if (t > c.ttime) return;
    if (fabs(c.target - c.start) < kEps) return;
    const double mt = c.ttime * (speed - c.start) / (c.target - c.start);
    c.shift = t - mt;
}
// sc_override with r ~ 1 / (target - start) (ppm::div_rcp): the same quotient. kChecked = false:
// operands known in range (k_prep's speed/time check); a zero quotient's sign cannot matter here
// (shift = t - mt).
template <bool kChecked = true>
__device__ __forceinline__ void sc_override_r(SC& c, double t, double speed, double r) {
    if (!kChecked) {      // the two early returns as a select (r = 1/(target - start) may be inf)
        const double mt = ppm::div_rcp_nc(c.ttime * (speed - c.start), c.target - c.start, r);
        const bool keep = t > c.ttime || fabs(c.target - c.start) < kEps;
        c.shift = keep ? c.shift : t - mt;
        return;
    }
    if (t > c.ttime) return;
    if (fabs(c.target - c.start) < kEps) return;
    const double mt = kChecked ? ppm::div_rcp(c.ttime * (speed - c.start), c.target - c.start, r)
                               : ppm::div_rcp_nc(c.ttime * (speed - c.start), c.target - c.start, r);
    c.shift = t - mt;
}

// k_cand<false>'s unchecked reciprocal divisions need every speed and ramp time of the scene's
// candidates to be +0 or of magnitude in [2^-60, 2^20] (LimitSpeed targets may be negative): every
// speed of a walk is then +0 or of magnitude in [2^-113, 2^21], every numerator of those
// divisions inside [2^-400, 2^400]
__device__ __forceinline__ bool speed_in_range(double x) {
    return x == 0 ? !__builtin_signbit(x) : (fabs(x) >= 0x1p-60 && fabs(x) <= 0x1p20);
}

// LimitSpeed::calculate (src/main.cpp:1068-1150). Returns 0 FREEFLOW 1 BRAKE 2 MAXBRAKE 3 ADJUST 4 KEEP.
__device__ inline int limit_speed(const pp_params& P, double fvx, double fvy, double next_s,
                                  double ego_s, double ego_speed, double ego_acc, bool in_lane,
                                  double& ts, double& tt, bool& collision) {
    int code = 0;
    bool can_acc = true;
    ts = P.max_speed;
    tt = fabs(ego_speed - P.max_speed) / P.relaxed_acc;
    double fcd = next_s - ego_s - P.car_length;
    collision = false;
    if (fcd < 0) { fcd = 0; collision = true; }
    const double fcs = sqrt(fvx * fvx + fvy * fvy);
    if (ego_speed > fcs) {
        double acc = P.relaxed_acc;
        if (ego_acc < 0) acc = P.min_relaxed_acc_while_braking;
        const double dv = ego_speed - fcs;
        const double dt = dv / acc;
        const double dd = ego_speed * dt - dv / 2 * dt;
        const double max_dist = fcd - P.safety_distance;
        if (dd > max_dist) {
            ts = fcs;
            tt = max_dist / (ego_speed - dv / 2);
            if (tt < kEps || dv / tt > P.maximum_acc) { code = 2; tt = dv / P.maximum_acc; }
            else code = 1;
            can_acc = false;
        }
    }
    if (can_acc && in_lane) {
        const double excess = ego_s + P.car_length + P.keep_distance - next_s;
        const double t_opt = s_min(1.0, fabs(excess) / 1.0);
        if (ego_s + P.car_length + P.keep_distance > next_s) {
            ts = fcs - excess / t_opt;
            tt = t_opt;
            const double mt = fabs(ts - ego_speed) / P.relaxed_acc;   // maximize_acc :1059-1067
            if (tt < mt) tt = mt;
            code = 3;
        } else if (ego_s + P.car_length + P.keep_distance + P.keep_distance_leeway > next_s) {
            ts = fcs;
            tt = 1.0;
            const double mt = fabs(ts - ego_speed) / P.relaxed_acc;
            if (tt < mt) tt = mt;
            code = 4;
        }
    }
    return code;
}

__device__ __forceinline__ uint32_t limit_flag(int code) {
    return code == 1 ? PP_ST_BRAKE : code == 2 ? PP_ST_MAXBRAKE : code == 3 ? PP_ST_ADJUST
         : code == 4 ? PP_ST_KEEP : 0u;
}

// candidate speed grid: k = 0 -> max_speed, else clamp(ego_speed + offset, 0, max_speed)
__device__ __forceinline__ double cand_speed(const pp_params& P, double ego_speed, int k) {
    if (k == 0) return P.max_speed;
    double v = ego_speed + P.speed_offsets[k - 1];
    if (v < 0) v = 0;
    if (v > P.max_speed) v = P.max_speed;
    return v;
}

}  // namespace ppd

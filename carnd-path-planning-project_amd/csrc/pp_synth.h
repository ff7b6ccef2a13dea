// pp_synth.h — deterministic synthetic scene generator (SURVEY.md §8(d) "Synthetic inputs").
//
// One counter-based Philox4x32-10 stream per scene (key = seed, counter = global scene index), so
// a scene depends only on (seed, index): identical on every GPU count and shard layout, and on the
// host. Only +, -, *, / on precomputed map tables are used (plus one atan2 for the telemetry yaw),
// so host and device outputs are bit-identical except ego_yaw_deg.
//
// Scene model (a highway snapshot around the ego):
//   ego on lane r (of PP_NUM_LANES) at a uniform point of the 181-waypoint loop, |d jitter| <= 0.3 m, speed U[0, 22.2]
//   (5 %: U[0, 3]), longitudinal accel U(-3, 3), 30 % of scenes drift laterally (U(-2, 2) m/s);
//   previous path = 10 points behind the ego along its lane, spacing v/50 (p9 = ego);
//   1 % of scenes are "frame 0" (n_prev = 0, telemetry pose only);
//   prev_target_lane = ego lane, 20 % an adjacent lane;
//   12 cars, ids 0..11, ds ~ U(-60, 250) m along their lane (2 %: half a loop away, usually
//   unmatchable), lane U{0..PP_NUM_LANES-1}, d jitter +-0.3, speed U(5, 25) along the lane tangent, vd ~ N(0, 0.3).
#pragma once
#include <stdint.h>
#include <math.h>

#include "pp_glibcm.h"

#ifndef PP_HD
#define PP_HD __host__ __device__
#endif
#ifndef PP_NUM_LANES
#define PP_NUM_LANES 3
#endif

namespace ppsynth {

// Precomputed lane polylines (host: pp_map_create; device: uploaded copy).
struct LaneTables {
    int n;                  // waypoints
    const double* lc_x;     // [lane * n + i] lane-center of waypoint i
    const double* lc_y;
    const double* seg_len;  // [lane * n + i] |lc[i] - lc[i-1]| (segment i ends at waypoint i)
    const double* tan_x;    // [lane * n + i] (lc[i] - lc[i-1]) / seg_len
    const double* tan_y;
};

// a ^ b ^ c: one v_bitop3_b32 on gfx950 (truth table 0x96), which the compiler does not form itself
#ifndef PP_BITOP3
#define PP_BITOP3 1
#endif
PP_HD inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__) && PP_BITOP3
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

PP_HD inline void philox_round(uint32_t ctr[4], const uint32_t key[2]) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = xor3(hi1, ctr[1], key[0]);
    const uint32_t n2 = xor3(hi0, ctr[3], key[1]);
    ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
}

// Philox4x32-10 block: counter (scene index lo/hi, block number, 0), key = seed.
PP_HD inline void philox4x32(uint64_t seed, uint64_t scene, uint32_t block, uint32_t out[4]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)scene, (uint32_t)(scene >> 32), block, 0x5EED0001u};
    for (int r = 0; r < 10; r++) {
        philox_round(ctr, key);
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
    out[0] = ctr[0]; out[1] = ctr[1]; out[2] = ctr[2]; out[3] = ctr[3];
}

// Monte-Carlo sensor noise (include/pp.h pp_mc_gauss): Irwin-Hall of four 32-bit uniforms of one
// Philox block, counter {scene, (draw * PP_NOISE_CAR_STRIDE + car) * 4 + q, 0x4D43}; unit variance; exactly rounded
// arithmetic only, so host and device agree bit for bit.
static_assert(PP_MAX_CARS <= PP_NOISE_CAR_STRIDE, "noise counter stride below the car limit");
#ifndef PP_IH_SUM
#define PP_IH_SUM 1
#endif
// the Irwin-Hall sum of one Philox block's words, as (s - 2) sqrt(3) (mc_gauss)
PP_HD inline double ih_unit(const uint32_t c[4]) {
    // (s - 2) sqrt(3) with s = sum_i (c_i + 0.5) 2^-32: every partial sum of that s is exact (at most
    // 35 significant bits), so s - 2 = (c_0 + c_1 + c_2 + c_3 - (2^33 - 2)) 2^-32 exactly; the
    // integer sum is exact in doubles too, and scaling sqrt(3) by 2^-32 is exact: the one rounding
    // left is the same product's
#if PP_IH_SUM
    const double t = (((double)c[0] + (double)c[1]) + ((double)c[2] + (double)c[3])) - 8589934590.0;
    return t * (1.7320508075688772 * 0x1p-32);
#else
    const double k = 1.0 / 4294967296.0;
    double s = ((double)c[0] + 0.5) * k;
    s += ((double)c[1] + 0.5) * k;
    s += ((double)c[2] + 0.5) * k;
    s += ((double)c[3] + 0.5) * k;
    return (s - 2.0) * 1.7320508075688772;
#endif
}
PP_HD inline double mc_gauss(uint64_t seed, uint64_t scene, int draw, int car, int q) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)scene, (uint32_t)(scene >> 32), (uint32_t)(((draw * PP_NOISE_CAR_STRIDE) + car) * 4 + q), 0x4D43u};
    for (int r = 0; r < 10; r++) {
        philox_round(ctr, key);
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
    return ih_unit(ctr);
}
// the four draws of one car (q = 0..3: x, y, vx, vy noise) at once: the same four Philox blocks as
// four mc_gauss calls, their rounds interleaved (independent chains)
PP_HD inline void mc_gauss4(uint64_t seed, uint64_t scene, int draw, int car, double g[4]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4][4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        ctr[q][0] = (uint32_t)scene; ctr[q][1] = (uint32_t)(scene >> 32);
        ctr[q][2] = (uint32_t)(((draw * PP_NOISE_CAR_STRIDE) + car) * 4 + q); ctr[q][3] = 0x4D43u;
    }
#pragma unroll
    for (int r = 0; r < 10; r++) {
#pragma unroll
        for (int q = 0; q < 4; q++) philox_round(ctr[q], key);
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) g[q] = ih_unit(ctr[q]);
}

struct Rng {
    uint64_t seed, scene;
    uint32_t block;
    uint32_t buf[4];
    int used;
    PP_HD Rng(uint64_t s, uint64_t sc) : seed(s), scene(sc), block(0), used(4) {}
    PP_HD uint32_t next() {
        if (used == 4) { philox4x32(seed, scene, block++, buf); used = 0; }
        return buf[used++];
    }
    // uniform in [0, 1): 53 random bits
    PP_HD double uni() {
        const uint32_t a = next() >> 5, b = next() >> 6;
        return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
    }
    PP_HD double uni(double lo, double hi) { return lo + (hi - lo) * uni(); }
    // approximately standard normal (Irwin-Hall, 4 uniforms): basic arithmetic only
    PP_HD double gauss() {   // sequenced: the call order must not depend on the compiler
        double s = uni();
        s += uni();
        s += uni();
        s += uni();
        return (s - 2.0) * 1.7320508075688772;
    }
    PP_HD int below(int k) { return (int)(uni() * k); }
};

// Walk `dist` metres (signed) along lane `lane` from segment `seg` (1..n; segment i ends at wp i)
// at fraction t. Returns the point and the segment tangent at the arrival point.
PP_HD inline void lane_walk(const LaneTables& T, int lane, int seg, double t, double dist,
                            double* px, double* py, double* ux, double* uy,
                            int* oseg = nullptr, double* ot = nullptr) {
    const int n = T.n;
    int i = seg;
    for (int it = 0; it < 4 * n + 8; it++) {
        const double L = T.seg_len[lane * n + i];
        if (dist >= 0) {
            const double rem = (1.0 - t) * L;
            if (dist <= rem || it == 4 * n + 7) { t = t + dist / L; break; }
            dist -= rem; t = 0.0; i = (i + 1 == n) ? 0 : i + 1;
        } else {
            const double rem = t * L;
            if (-dist <= rem || it == 4 * n + 7) { t = t + dist / L; break; }
            dist += rem; t = 1.0; i = (i == 0) ? n - 1 : i - 1;
        }
    }
    const int ip = (i == 0) ? n - 1 : i - 1;
    const double ax = T.lc_x[lane * n + ip], ay = T.lc_y[lane * n + ip];
    const double bx = T.lc_x[lane * n + i], by = T.lc_y[lane * n + i];
    *px = ax + (bx - ax) * t;
    *py = ay + (by - ay) * t;
    *ux = T.tan_x[lane * n + i];
    *uy = T.tan_y[lane * n + i];
    if (oseg) { *oseg = i; *ot = t; }
}

// The rollout simulator's traffic (include/pp.h pp_traffic): car j of scene s at [j * S + s].
struct TrafficV {
    int64_t S;
    int n;
    int32_t *lane, *seg;
    double *t, *off, *v;
};

// Car on lane `lane` at fraction t of segment `seg`, lateral offset `off`, speed v along the lane:
// telemetry position and velocity (the same formulas as synth_scene's cars, lateral speed 0).
PP_HD inline void traffic_car(const LaneTables& T, int lane, int seg, double t, double off, double v,
                              double* x, double* y, double* vx, double* vy) {
    const int n = T.n;
    const int ip = (seg == 0) ? n - 1 : seg - 1;
    const double ax = T.lc_x[lane * n + ip], ay = T.lc_y[lane * n + ip];
    const double bx = T.lc_x[lane * n + seg], by = T.lc_y[lane * n + seg];
    const double px = ax + (bx - ax) * t, py = ay + (by - ay) * t;
    const double ux = T.tan_x[lane * n + seg], uy = T.tan_y[lane * n + seg];
    *x = px + uy * off;
    *y = py - ux * off;
    *vx = ux * v;
    *vy = uy * v;
}

// Advance (seg, t) by dist >= 0 metres along the lane polyline (lane_walk's forward branch).
PP_HD inline void lane_advance(const LaneTables& T, int lane, int* seg, double* t, double dist) {
    const int n = T.n;
    int i = *seg;
    double tt = *t;
    for (int it = 0; it < 4 * n + 8; it++) {
        const double L = T.seg_len[lane * n + i];
        const double rem = (1.0 - tt) * L;
        if (dist <= rem || it == 4 * n + 7) { tt = tt + dist / L; break; }
        dist -= rem; tt = 0.0; i = (i + 1 == n) ? 0 : i + 1;
    }
    *seg = i;
    *t = tt;
}

// Writable view of one batch (pointers into SoA arrays, see include/pp.h index conventions).
struct OutBatch {
    int64_t S;
    double *ego_x, *ego_y, *ego_yaw_deg, *ego_speed_mph, *prev_x, *prev_y;
    int32_t *n_prev, *prev_target_lane, *n_cars, *car_id;
    double *car_x, *car_y, *car_vx, *car_vy;
};

constexpr int kSynthCars = 12;

// Generates scene `local` of the batch from global index `g`. yaw uses atan2 (the one
// transcendental); everything else is exact arithmetic on the lane tables.
PP_HD inline void synth_scene(const LaneTables& T, uint64_t seed, int64_t g, int64_t local,
                              const OutBatch& o, const TrafficV* traffic = nullptr) {
    Rng r(seed, (uint64_t)g);
    const int64_t S = o.S;
    const int n = T.n;
    const int seg = r.below(n);
    const double t = r.uni();
    const int lane = r.below(PP_NUM_LANES);
    const double djit = r.uni(-0.3, 0.3);
    double v = r.uni(0.0, 22.2);
    if (r.uni() < 0.05) v = r.uni(0.0, 3.0);
    const double acc = r.uni(-3.0, 3.0);
    const double vd_lat = (r.uni() < 0.3) ? r.uni(-2.0, 2.0) : 0.0;
    const bool frame0 = r.uni() < 0.01;
    int ptl = lane;
    if (r.uni() < 0.2) {
        const int dir = (r.uni() < 0.5) ? -1 : 1;
        ptl = lane + dir;
        if (ptl < 0 || ptl > PP_NUM_LANES - 1) ptl = lane - dir;
    }
    // previous path: p9 = ego; p_{9-k} walked back sum_{m<k} spacing_m along the lane
    double back = 0.0;
    double ex = 0, ey = 0, eux = 1, euy = 0;
    for (int k = 0; k < 10; k++) {
        double px, py, ux, uy;
        lane_walk(T, lane, seg, t, -back, &px, &py, &ux, &uy);
        const double dk = djit - vd_lat * k * 0.02;   // lateral offset k steps in the past
        // right-hand normal (Map::Init convention: n = (dy, -dx) / len)
        const double qx = px + uy * dk, qy = py - ux * dk;
        o.prev_x[(int64_t)(9 - k) * S + local] = qx;
        o.prev_y[(int64_t)(9 - k) * S + local] = qy;
        if (k == 0) { ex = qx; ey = qy; eux = ux; euy = uy; }
        double sp = v - acc * (k + 1) * 0.02;
        if (sp < 0.0) sp = 0.0;
        back += sp / 50.0;
    }
    o.ego_x[local] = ex;
    o.ego_y[local] = ey;
    o.ego_yaw_deg[local] = ppg::atan2(euy, eux) * 180.0 / 3.14159265358979323846;   // glibc's, host == device
    o.ego_speed_mph[local] = v * 2.237;
    o.n_prev[local] = frame0 ? 0 : 10;
    o.prev_target_lane[local] = ptl;
    o.n_cars[local] = kSynthCars;
    for (int j = 0; j < kSynthCars; j++) {
        const int64_t ix = (int64_t)j * S + local;
        double ds = r.uni(-60.0, 250.0);
        if (r.uni() < 0.02) ds = 0.5 * 6945.554;
        const int cl = r.below(PP_NUM_LANES);
        const double cd = r.uni(-0.3, 0.3);
        const double cs = r.uni(5.0, 25.0);
        const double cvd = 0.3 * r.gauss();
        double px, py, ux, uy;
        int cseg;
        double ct;
        lane_walk(T, cl, seg, t, ds, &px, &py, &ux, &uy, &cseg, &ct);
        if (traffic) {
            const int64_t tx = (int64_t)j * traffic->S + local;
            traffic->lane[tx] = cl; traffic->seg[tx] = cseg; traffic->t[tx] = ct;
            traffic->off[tx] = cd; traffic->v[tx] = cs;
        }
        o.car_id[ix] = j;
        o.car_x[ix] = px + uy * cd;
        o.car_y[ix] = py - ux * cd;
        o.car_vx[ix] = ux * cs + uy * cvd;
        o.car_vy[ix] = uy * cs - ux * cvd;
    }
}

}  // namespace ppsynth

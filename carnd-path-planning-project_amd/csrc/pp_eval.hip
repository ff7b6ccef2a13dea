// pp_eval.hip — MI355X (gfx950) batched trajectory-candidate evaluator + its C-ABI.
//
// Pipeline per pp_eval call:
//   K1 k_prep    one lane per scene, map staged in LDS: ego derivation, Frenet frame, car matching,
//                LaneChangePlanner, follow cars + LimitSpeed per candidate lane
//                (src/main.cpp:1254-1438) -> per-scene prep record (SoA workspace).
//   K2 k_cand    one workgroup = SPB scenes x C candidates. Phase A: one lane per (scene, lane)
//                builds the control points + tk::spline coefficients into LDS
//                (TrajectoryBuilder::build setup, src/main.cpp:575-904, spline.h:284-373).
//                Phase B: one lane per candidate runs the 0.02 s resampling loop with the
//                accel/curvature limiter (src/main.cpp:905-1041) reading its spline from LDS
//                and computes the candidate cost (cost-only loop unless every path is emitted).
//   K3 k_winner  comfort mode: per-scene argmin + re-run of the winning candidate with outputs.
//                (reference mode: the winner is known before the loop; k_cand's first wave of
//                each block runs the winners and writes next_x/next_y)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/pp.h"
#include "pp_cartable.h"
#if defined(PP_DIAG) || defined(PP_LIMCENSUS)
// diagnostic builds only (-DPP_DIAG, -DPP_LIMCENSUS): per event, [2k] lanes where it fired,
// [2k+1] waves where any lane fired (the wave executes the branch). Read with pp_diag_read.
constexpr int kDiagWords = 96;
__device__ unsigned long long g_diag[kDiagWords];
__device__ __forceinline__ void diag(int k, bool c) {
    const unsigned long long b = __ballot(c);
    if (b && __lane_id() == (unsigned)__builtin_ctzll(__ballot(1))) {
        atomicAdd(&g_diag[2 * k], (unsigned long long)__builtin_popcountll(b));
        atomicAdd(&g_diag[2 * k + 1], 1ull);
    }
}
#endif
#ifdef PP_DIAG
#define PP_DIAGC(k, c) diag(k, c)
#else
#define PP_DIAGC(k, c) ((void)0)
#endif
// The limiter census (-DPP_LIMCENSUS; VERDICT r5 item 2, tests/test_full_batch.py): at every
// decision of the acceleration limiter (src/main.cpp:941 and :972) the census build also evaluates
// the reference's own operation sequence from the same state — the speed ramp's IEEE division,
// glibc's atan2 of the step (pp_glibcm.h, bit for bit) and the wrapped difference of absolute
// angles — and counts decisions within a relative 1e-12 of maximum_acc and decisions the two
// sequences take differently (g_diag events 26-33, names in tests/test_full_batch.py).
#ifdef PP_LIMCENSUS
#define PP_CEN(k, c) diag(k, c)
#else
#define PP_CEN(k, c) ((void)0)
#endif
#ifdef PP_CENSUS
// census builds only (-DPP_CENSUS): an assembly comment ";@R <output mode> <region>" at the start of
// each region of the candidate loop; tools/valu_census.py counts each region's instructions in the
// build's ISA and multiplies them by how often a wave executes the region (tools/diag_events.py)
#define PP_REGION(name) asm volatile(";@R %0 " name ::"i"(kOutMode))
#define PP_REGION_K(name) asm volatile(";@R 7 " name)
#define PP_REGION_A(name) asm volatile(";@R 8 " name)
#else
#define PP_REGION_A(name) ((void)0)
#define PP_REGION(name) ((void)0)
#define PP_REGION_K(name) ((void)0)
#endif
#ifdef PP_CHECK
// checking builds only (-DPP_CHECK): every global store of k_cand / k_emit (and the record reads
// of k_emit) is tested against the buffer it belongs to, and k_cand poisons its LDS slots at the
// start of every group, so a slot read that phase A of the same group did not write shows up as a
// NaN result or a meta sentinel. g_chk: [0] violations, [1] first site, [2] its offset, [3] its
// workgroup, [4] its group. Read with pp_check_read.
struct ChkLim {
    const double *paths, *nx, *ny, *rec, *cost;
    const unsigned long long* adjm;
    long long npaths, nnext, nrec, nadj, ncost, nscen;
};
__device__ unsigned long long g_chk[8];
__device__ ChkLim g_lim;
__device__ __forceinline__ bool chk_(bool ok, int site, long long off, long long grp) {
    if (!ok && atomicAdd(&g_chk[0], 1ull) == 0ull) {
        g_chk[1] = (unsigned long long)site; g_chk[2] = (unsigned long long)off;
        g_chk[3] = blockIdx.x; g_chk[4] = (unsigned long long)grp;
    }
    return ok;
}
// p inside [g_lim.B, g_lim.B + g_lim.N)
#define PP_CHKP(p, B, N, site) chk_((const void*)(p) >= (const void*)g_lim.B && (const void*)(p) < (const void*)(g_lim.B + g_lim.N), site, (long long)((const char*)(p) - (const char*)g_lim.B), -1)
#define PP_CHK(ok, site, off) chk_((ok), site, (long long)(off), -1)
constexpr int kMetaPoison = 0x7fffffff;
#else
#define PP_CHKP(p, B, N, site) true
#define PP_CHK(ok, site, off) true
#endif
#ifdef PP_TRACE
// diagnostic builds only (-DPP_TRACE): per workgroup of the traced kernel (k_cand<false>, and k_prep
// at kTraceK1 + blockIdx), 8 words: [0] start, [1] end of phase A, [2..5] end of phase B per wave,
// [6] end, [7] XCC id << 32 | HW_ID; times from the 100 MHz constant clock. Read with pp_trace_read.
constexpr int kTraceMax = 1 << 18, kTraceK1 = 3 << 16;
__device__ unsigned long long g_trace[8 * kTraceMax];
__device__ __forceinline__ void trace_at(unsigned long long blk, int k) {   // blk < kTraceMax
    g_trace[8 * blk + k] = wall_clock64();
}
__device__ __forceinline__ unsigned long long trace_hwid() {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));    // HW_REG_XCC_ID
    return ((unsigned long long)xcc << 32) | hw;
}
#define PP_TRACE_AT(blk, k) do { if ((blk) < (unsigned)kTraceK1) trace_at((blk), (k)); } while (0)
// the grouped K1 of block 0 (k_step_small's single frame), lane 0: words at group kTraceK1 - 2
#define PP_TRACE_K1(k) do { if (blockIdx.x == 0 && threadIdx.x == 0) trace_at(kTraceK1 - 2, (k)); } while (0)
#else
#define PP_TRACE_AT(blk, k) ((void)0)
#define PP_TRACE_K1(k) ((void)0)
#endif
#include "pp_device.h"
#include "pp_glibcm.h"
#include "pp_math.h"
#include "pp_synth.h"

using namespace ppd;


// ------------------------------------------------------------------------------------------------
// K1: scene preparation
// ------------------------------------------------------------------------------------------------
// kMapArrays arrays of n: ref_x ref_y nx ny lc_x[NL] lc_y[NL] llen[NL] lden[NL] lrcp[NL]
// atab: the approach table (global memory; build_atab; null: none); atab_lds: it fits k_prep<true,
// false>'s LDS after the map (that kernel stages it there: the host passes it only then)
struct MapG { const double* buf; int n; int fastm; WGrid wg; const double2* wseg; const double* atab; int atab_lds; };

// |angle| bound for the hot loop: the loop adds at most 2*pi per curvature adjustment over
// <= PP_MAX_POINTS steps, which keeps every sin/cos argument below ppm::kMediumMax.
constexpr double kSlowAngle = 1.0e5;
constexpr int kLimSlow = 1 << 7;   // internal bit in PrepV.lim_mask
static_assert(NL <= 6, "lim_mask: bit 0 in-lane limit, bits 1..NL lane limits, bit 7 kLimSlow");

__device__ __forceinline__ MapV map_view(const double* b, int n, int fastm = 0) {
    MapV m;
    m.ref_x = b; m.ref_y = b + n; m.nx = b + 2 * n; m.ny = b + 3 * n;
    m.lc_x = b + 4 * n; m.lc_y = b + (4 + NL) * n; m.llen = b + (4 + 2 * NL) * n;
    m.lden = b + (4 + 3 * NL) * n; m.lrcp = b + (4 + 4 * NL) * n; m.n = n; m.fastm = fastm;
    return m;
}

// The winner record (written once by k_cand, read once by k_emit), next_x/next_y (written once)
// and every emitted path point are nontemporal (streaming) accesses
#define PP_ST(p, v) __builtin_nontemporal_store((v), (p))
#define PP_LD(p) __builtin_nontemporal_load(p)
// one (x, y) path point: a 16-B store (p 16-B aligned: paths are [.., c] pairs of doubles)
__device__ __forceinline__ void st_xy(double* p, double x, double y) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    const dv2 xy = {x, y};
    __builtin_nontemporal_store(xy, (dv2*)p);
}
// ---- The output frame: the local -> global transform of TrajectoryBuilder::build (src/main.cpp:
// 786-823, 994-1007, 1033-1037). No decision of the loop reads it, so its turns (curvature
// adjustments) are evaluated in fused multiply-adds with an angle-sum rotation of the heading; every
// launch shape that writes the reference decision's next_x/next_y (k_emit, the fused small-batch
// kernels) or a winner's (k_winner) calls these same functions, so their outputs stay bit-identical
// to each other (and within ~1e-11 m of the reference after a turn, equal to it before the first
// one). k_cand's all-paths mode has a cheaper variant below (frame_pt_fma, frame_turn_at).
struct OutFrame { double cx, cy, ca, sa; };   // centre, cos and sin of the frame's heading
// a point: the reference's own operations (src/main.cpp:1033-1036), unfused: until a path's first
// curvature adjustment its points carry the reference's bits, and in a closed loop those first
// points are the next frame's previous path (its ego speed, heading and spline knots)
__device__ __forceinline__ void frame_pt(const OutFrame& f, double px, double py, double& ox, double& oy) {
    ox = (px * f.ca - py * f.sa) + f.cx;
    oy = (px * f.sa + py * f.ca) + f.cy;
}
// the turn of a curvature adjustment (src/main.cpp:986-997) at local point (px, py): the centre
// rotates about the current output point, the heading's (cos, sin) by the angle-sum rotation
__device__ __forceinline__ void frame_turn(OutFrame& f, double px, double py, double cr, double sr) {
    double tx, ty;
    frame_pt(f, px, py, tx, ty);
    const double vx = f.cx - tx, vy = f.cy - ty;
    f.cx = tx + __builtin_fma(vx, cr, -(vy * sr));
    f.cy = ty + __builtin_fma(vx, sr, vy * cr);
    const double nca = __builtin_fma(f.ca, cr, -(f.sa * sr)), nsa = __builtin_fma(f.sa, cr, f.ca * sr);
    f.ca = nca;
    f.sa = nsa;
}
// the turn angle rot = nad - adiff (src/main.cpp:978-986), nad = +-nc / speed / 50 with the sign of
// adiff: k_cand<false> (speed +0 or in [2^-113, 2^21]) by a reciprocal, the checked instantiation by
// IEEE divisions (speed 0: +-inf or NaN, which turns the rest of the path into NaN either way)
template <bool kLarge>
__device__ __forceinline__ double turn_angle(double nc, double speed, double adiff) {
    double nad = kLarge ? nc / speed / 50 : (nc * 0.02) * ppm::rcp_nr(speed);
    if (adiff < 0) nad *= -1;
    return nad - adiff;
}
// sin and cos of a turn: fdlibm's kernel polynomials in fused form (~1 ulp) on [-pi/4, pi/4]; a
// wider turn (rare: a wide step turn, or a step slower than ~0.7 m/s) is first reduced by the
// nearest multiple of pi/2 (two-part Cody-Waite: |error| < 1e-15 rad up to kMediumMax, plenty for an
// output frame) and its quadrant applied after; beyond kMediumMax (only from an absurd telemetry
// heading, in the checked instantiation) the library's reduction
// a constant materialised at its use (scalar moves) rather than hoisted out of the step loop into
// registers that the loop then holds throughout
__device__ __forceinline__ double kc(double v) {
    asm volatile("" : "+s"(v));
    return v;
}
template <bool kLarge>
__device__ __forceinline__ void turn_sincos(double r, double& s, double& c) {
    double y = r;
    int q = 0;
    if (__builtin_expect(!(fabs(r) <= 0.78539816339744828), 0)) {
        if (kLarge && !(fabs(r) <= ppm::kMediumMax)) {
            ppm::sincos_pp<true>(r, s, c);
            return;
        }
        const double k = __builtin_rint(r * 6.36619772367581382433e-01);
        y = __builtin_fma(-k, kc(1.57079632673412561417e+00), r);
        y = __builtin_fma(-k, kc(6.07710050650619224932e-11), y);
        q = (int)k;
    }
    const double z = y * y;
    double ps = __builtin_fma(z, kc(1.58969099521155010221e-10), kc(-2.50507602534068634195e-08));
    ps = __builtin_fma(z, ps, kc(2.75573137070700676789e-06));
    ps = __builtin_fma(z, ps, kc(-1.98412698298579493134e-04));
    ps = __builtin_fma(z, ps, kc(8.33333333332248946124e-03));
    ps = __builtin_fma(z, ps, kc(-1.66666666666666324348e-01));
    double pc = __builtin_fma(z, kc(-1.13596475577881948265e-11), kc(2.08757232129817482790e-09));
    pc = __builtin_fma(z, pc, kc(-2.75573143513906633035e-07));
    pc = __builtin_fma(z, pc, kc(2.48015872894767294178e-05));
    pc = __builtin_fma(z, pc, kc(-1.38888888888741095749e-03));
    pc = __builtin_fma(z, pc, kc(4.16666666666666019037e-02));
    s = __builtin_fma(y * z, ps, y);
    c = __builtin_fma(z * z, pc, __builtin_fma(-0.5, z, 1.0));
    if (__builtin_expect(q != 0, 0)) {
        if (q & 1) { const double t = s; s = c; c = -t; }
        if (q & 2) { s = -s; c = -c; }
    }
}

// k_cand's all-paths mode (output mode 4): the same output frame, cheaper. Every candidate writes
// its path there, so the point transform runs on every lane-step and a turn on about half of all
// wave-steps (for one lane in ten): each point is two fused multiply-adds per coordinate
// (frame_pt_fma); the loop keeps the last output point o, so a turn sets the centre from it — c = o -
// R' p, the current point keeps its output — instead of rotating the old centre about o; the turn
// angle's reciprocal takes one Newton step. ~1e-13 m from the shared turn (frame_turn); the paths' tolerance is 1e-6 m, and
// no decision and no closed loop reads these points (the reference decision's next_x/next_y and
// every fed-back path come from frame_turn / k_emit).
__device__ __forceinline__ void frame_turn_at(OutFrame& f, double px, double py, double ox, double oy,
                                              double cr, double sr) {
    const double nca = __builtin_fma(f.ca, cr, -(f.sa * sr)), nsa = __builtin_fma(f.sa, cr, f.ca * sr);
    f.ca = nca;
    f.sa = nsa;
    f.cx = ox - __builtin_fma(nca, px, -(nsa * py));
    f.cy = oy - __builtin_fma(nsa, px, nca * py);
}
__device__ __forceinline__ void frame_pt_fma(const OutFrame& f, double px, double py, double& ox, double& oy) {
    ox = __builtin_fma(px, f.ca, __builtin_fma(-py, f.sa, f.cx));
    oy = __builtin_fma(px, f.sa, __builtin_fma(py, f.ca, f.cy));
}
__device__ __forceinline__ double turn_angle_fast(double nc, double speed, double adiff) {
    double r = __builtin_amdgcn_rcp(speed);
    r = __builtin_fma(__builtin_fma(-speed, r, 1.0), r, r);
    double nad = (nc * 0.02) * r;          // (speed, hence nad, may be negative)
    if (adiff < 0) nad = -nad;
    return nad - adiff;
}
// Round 5 (PP_PATHS_INC, default on): k_cand's all-paths frame without a centre. The reference's
// turn rotates the centre about the current output point tp (src/main.cpp:995-1004), so tp stays
// where it is and every later point is o_{k+1} = o_k + R_{k+1} (p_{k+1} - p_k): the loop keeps the
// last output point o and the heading (ca, sa) only, and a point is o plus the rotated local step
// (frame_step: the same four fused multiply-adds as frame_pt_fma). A narrow turn (the step's
// angle came from asin(u_prev x u): |adiff| <= 0.0709) rotates by rot = nad - adiff, i.e. by
// R(nad) R(-adiff), and (cos, sin)(adiff) are the step's own unit-vector products (dt, cr): only
// sin/cos of |nad| < |adiff| are left, short Taylor polynomials (sincos_small). The points differ
// from the reference's by rounding only (the summed steps: ~1e-13 m over a 100-point path); no
// decision reads them.
#ifndef PP_PATHS_INC
#define PP_PATHS_INC 1
#endif
#ifndef PP_RCP1
#define PP_RCP1 0
#endif
#ifndef PP_DT_NARROW
#define PP_DT_NARROW 0
#endif

// a narrow step turn (asin_small's domain): u_prev . u > 0 and |u_prev x u| <= kStepSinMax; for unit
// vectors (to a few ulps) the same as u_prev . u >= sqrt(1 - kStepSinMax^2) (PP_DT_NARROW: one
// compare; |cr| then exceeds kStepSinMax by < 1e-14 at most, where the series is as accurate)
#if PP_DT_NARROW
#define PP_NARROW(dt, cr) ((dt) >= 0.99749053128338025)
#else
#define PP_NARROW(dt, cr) ((dt) > 0 && fabs(cr) <= ppm::kStepSinMax)
#endif
__device__ __forceinline__ void frame_step(double ca, double sa, double dpx, double dpy, double& ox, double& oy) {
    ox = __builtin_fma(dpx, ca, __builtin_fma(-dpy, sa, ox));
    oy = __builtin_fma(dpx, sa, __builtin_fma(dpy, ca, oy));
}
// sin and cos of |x| <= 0.0709: sin through x^7 (next term x^9/9! < 1.3e-16), cos through x^8 (next
// term x^10/10! < 1e-18)
__device__ __forceinline__ void sincos_small(double x, double& s, double& c) {
    const double z = x * x;
    double ps = __builtin_fma(z, kc(-1.98412698412698412698e-04), kc(8.33333333333333333333e-03));
    ps = __builtin_fma(z, ps, kc(-1.66666666666666666667e-01));
    s = __builtin_fma(x * z, ps, x);
    double pc = __builtin_fma(z, kc(2.48015873015873015873e-05), kc(-1.38888888888888888889e-03));
    pc = __builtin_fma(z, pc, kc(4.16666666666666666667e-02));
    pc = __builtin_fma(z, pc, -0.5);
    c = __builtin_fma(z, pc, 1.0);
}
// the heading turned by (cr, sr) = (cos, sin) of the rotation
__device__ __forceinline__ void frame_rot(double& ca, double& sa, double cr, double sr) {
    const double nca = __builtin_fma(ca, cr, -(sa * sr)), nsa = __builtin_fma(sa, cr, ca * sr);
    ca = nca;
    sa = nsa;
}
// a narrow turn: nad = +-nc / speed / 50 with adiff's sign (src/main.cpp:983-984; adiff is never
// -0: x - pi rounds an exact cancellation to +0), (cos, sin)(rot) = R(nad) applied to (dt, -cr)
__device__ __forceinline__ void turn_narrow(double& ca, double& sa, double nc, double speed, double adiff,
                                            double dt, double cr) {
    double r = __builtin_amdgcn_rcp(speed);
    r = __builtin_fma(__builtin_fma(-speed, r, 1.0), r, r);
    const double nad = __builtin_copysign((nc * 0.02) * r, adiff);
    double sn, cn;
    sincos_small(nad, sn, cn);
    frame_rot(ca, sa, __builtin_fma(cn, dt, sn * cr), __builtin_fma(sn, dt, -(cn * cr)));
}
// Tuning constants (each measured against its alternatives):
#ifndef PP_EMIT_CHUNK
#define PP_EMIT_CHUNK 4
#endif
constexpr int kEmitChunk = PP_EMIT_CHUNK;   // emit_scene_pre (small batches): recorded steps loaded together per lane
constexpr int kEmitRows = 8;       // k_emit (large batches, emit_scene_rows): output rows per load round
constexpr int kWalkPf = 4;         // segments of the control-point walk loaded ahead (get_lane_pos_fwd)
constexpr int kPrepWaves = 3;      // k_prep waves per SIMD (kW4: 4)
#ifndef PP_CAND_WAVES
#define PP_CAND_WAVES 4
#endif
#ifndef PP_CAND_WAVES2
#define PP_CAND_WAVES2 PP_CAND_WAVES    // the all-paths instantiation k_cand<., 2>
#endif
#ifndef PP_UNROLL2
#define PP_UNROLL2 1
#endif
#ifndef PP_ASIN_S
#define PP_ASIN_S 0
#endif
constexpr int kCandWaves = PP_CAND_WAVES;   // k_cand waves per SIMD (<= 128 VGPRs)
// Winner record (k_cand -> k_emit), room = N - K steps of scene s, rstride = room S: point-major
// arrays, pos_x at rec[g S + s], pos_y at rec[rstride + g S + s], the rotation of an adjusted step
// at rec[2 rstride + g S + s] (every address of scene s is = s mod S: a wave's accesses coalesce)
__device__ __forceinline__ double* rec_px(double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s) {
    (void)rstride;
    return rec + g * S + s;
}
__device__ __forceinline__ double* rec_py(double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s) {
    return rec + rstride + g * S + s;
}
__device__ __forceinline__ double* rec_rot(double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s) {
    return rec + 2 * rstride + g * S + s;
}
__device__ __forceinline__ const double* rec_rot(const double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s) {
    return rec_rot((double*)rec, rstride, g, S, s);
}
__device__ __forceinline__ void rec_st(double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s,
                                       double x, double y) {
    PP_ST(rec_px(rec, rstride, g, S, s), x);
    PP_ST(rec_py(rec, rstride, g, S, s), y);
}
__device__ __forceinline__ void rec_ld(const double* rec, int64_t rstride, int64_t g, int64_t S, int64_t s,
                                       double& x, double& y) {
    double* r = (double*)rec;
    x = PP_LD(rec_px(r, rstride, g, S, s));
    y = PP_LD(rec_py(r, rstride, g, S, s));
}
// The map into LDS (16-B aligned both sides): 16-B loads, each thread's loads issued before its LDS
// stores, so a block stages a map of up to 8 x 512 doubles (highway_map.csv: 3,439) in one round
// trip to memory instead of one per element (the single-frame kernel waits for it)
__device__ __forceinline__ void stage_map(double* __restrict__ dst, const double* __restrict__ src, int nd) {
    typedef double dv2 __attribute__((ext_vector_type(2)));
    constexpr int kU = 8;
    const int n2 = nd / 2;
    for (int i0 = threadIdx.x; i0 < n2; i0 += kU * blockDim.x) {
        dv2 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * (int)blockDim.x;
            if (i < n2) v[u] = ((const dv2*)src)[i];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * (int)blockDim.x;
            if (i < n2) ((dv2*)dst)[i] = v[u];
        }
    }
    if ((nd & 1) && threadIdx.x == 0) dst[nd - 1] = src[nd - 1];
}
// kLdsMap: the map (kMapArrays n doubles) is staged in LDS (n <= kLdsMapMax: <= 62.4 KB, 600
// waypoints at three lanes); larger maps are read from global memory (L2-resident) by the same code.
constexpr int kLdsMapMax = 62400 / (8 * kMapArrays);

// the velocity k_prep's car pass used for the car of iteration index it (src/main.cpp:1343-1346):
// the table slot it (written or stale) with a car table, else row it plus its Monte-Carlo noise
__device__ __forceinline__ void car_velocity(const pp_scene_batch& in, const pp_params& P, int64_t S,
                                             int64_t s, int draw, bool tab, int it, double& vx, double& vy) {
    const int64_t ix = (int64_t)it * S + s;
    if (tab) { vx = in.tab_vx[ix]; vy = in.tab_vy[ix]; return; }
    vx = in.car_vx[ix]; vy = in.car_vy[ix];
    if (draw > 0) {
        const uint64_t gs = (uint64_t)(P.noise_first_scene + s);
        vx += P.noise_vel_sigma * ppsynth::mc_gauss(P.noise_seed, gs, draw, it, 2);
        vy += P.noise_vel_sigma * ppsynth::mc_gauss(P.noise_seed, gs, draw, it, 3);
    }
}
// k_cand groups (SPB scenes per group, or BPS groups per scene): k_prep marks the groups holding a
// kLimSlow scene in this bitmap for k_cand<true>
// (list/count: the flagged groups in the order k_prep found them, for k_cand<true>; count is zeroed
// before every K1)
// (BPS < 0: the flat all-paths geometry, groups of 256 consecutive candidates of the batch, C per
// scene: a scene lies in groups s C / 256 ... ((s + 1) C - 1) / 256)
struct GroupBits { uint32_t* bits; int SPB, BPS; uint32_t* list; uint32_t* count; int pose_by_wave; int C; };
// ---- K1 building blocks, shared by k_prep (one lane per evaluation) and k_prep_g2..16 (G lanes) ----

// Ego state of one evaluation: derivation (src/main.cpp:1233-1292), Frenet frame and ego matching
// (:1299-1320).
struct EgoSt {
    double ego_x, ego_y, yaw, ego_speed, ego_acc, esv_x, esv_y, dt0, p8x, p8y;
    double ego_s, ego_d, ego_vs, ego_vd, ratio[NL];
    int K, ref_wp, ego_lane;
    uint32_t status;
};

// G > 1: the G lanes of a group (this one is lane r) split the reference-waypoint scan; every
// lane ends with the same state
template <int G>
__device__ __forceinline__ void prep_ego(const MapV& m, const pp_scene_batch& in, const pp_params& P,
                                         int64_t S, int64_t s, int r, EgoSt& e) {
    e.status = 0;
    e.ego_x = in.ego_x[s]; e.ego_y = in.ego_y[s];
    e.yaw = in.ego_yaw_deg[s];
    double ego_speed = in.ego_speed_mph[s];
    ego_speed /= 2.237;
    e.ego_acc = 0; e.esv_x = 0; e.esv_y = 0; e.dt0 = 0;
    e.K = 0;
    e.p8x = 0; e.p8y = 0;
    // (the kept points are loaded with n_prev, not after it: rows 7-9 always exist, and a frame's
    // K1 would otherwise wait for two memory round trips in a row)
    const int np = in.n_prev[s];
    const double p7x = in.prev_x[7 * S + s], p7y = in.prev_y[7 * S + s];
    const double p8x = in.prev_x[8 * S + s], p8y = in.prev_y[8 * S + s];
    const double p9x = in.prev_x[9 * S + s], p9y = in.prev_y[9 * S + s];
    if (np >= PP_PREV_KEEP) {
        e.K = PP_PREV_KEEP;
        e.p8x = p8x; e.p8y = p8y;
        const double ax = e.p8x - p7x, ay = e.p8y - p7y;
        const double v2 = sqrt(ax * ax + ay * ay);
        e.esv_x = p9x - e.p8x; e.esv_y = p9y - e.p8y;
        const double v3 = sqrt(e.esv_x * e.esv_x + e.esv_y * e.esv_y);
        e.ego_acc = (v3 - v2) * 50;
        ego_speed = v3 * 50;
        e.esv_x *= 50; e.esv_y *= 50;
        e.ego_x = p9x; e.ego_y = p9y;
        e.dt0 = PP_PREV_KEEP / 50.0;
    }
    e.ego_speed = ego_speed;
    if (G == 1) init_reference_waypoint(m, e.ego_x, e.ego_y, e.ref_wp, e.ratio);
    else init_reference_waypoint_grp<G>(m, e.ego_x, e.ego_y, r, e.ref_wp, e.ratio);
    e.ego_s = 0; e.ego_d = 0;
    e.ego_lane = 0;
    int nwp_unused = 0;
    if (!lane_match(m, e.ref_wp, e.ratio, e.ego_x, e.ego_y, e.ego_s, e.ego_d, e.ego_lane, nwp_unused)) {
        e.ego_s = e.ego_d = 0;
        e.ego_lane = 0;
        e.status |= PP_ST_EGO_UNMATCHED;
    }
    project_speed(m, e.esv_x, e.esv_y, e.ref_wp, e.ego_vs, e.ego_vd);
    if (e.ego_acc > P.maximum_acc) e.ego_acc = P.maximum_acc;
    if (e.ego_acc < -P.maximum_acc) e.ego_acc = -P.maximum_acc;
}

// LaneChangePlanner's accumulation (src/main.cpp:377-445) and the follow-car selection
// (:1388-1410): order-dependent reductions over one car sequence. Every one is a minimum with ties
// to the lower iteration index (or an AND / a count), so a visiting order other than ascending
// ids gives the reference's result once ties compare that index explicitly — except for a chosen
// car whose id is the reference's 'no car' sentinel -1, which any later car replaces: such
// scenes (and car tables) are visited in iteration order.
// (Per-lane state is indexed by the car's lane through selects, sel/put: a dynamically indexed
// member array would live in scratch memory.)
// (each element passes an empty asm first: a select chain over the array's own elements is
// folded back into an indexed load, which puts the array in scratch memory)
template <typename T>
__device__ __forceinline__ T sel(const T (&a)[NL], int l) {
    T x = a[0];
    asm("" : "+v"(x));
#pragma unroll
    for (int i = 1; i < NL; i++) {
        T ai = a[i];
        asm("" : "+v"(ai));
        x = l == i ? ai : x;
    }
    return x;
}
template <typename T>
__device__ __forceinline__ void put(T (&a)[NL], int l, T x) {
#pragma unroll
    for (int i = 0; i < NL; i++) a[i] = l == i ? x : a[i];
}
// OR / sum over the G lanes of a group; (key, index) minimum with ties to the lower index
template <int G>
__device__ __forceinline__ uint32_t grp_or(uint32_t x) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) x |= (uint32_t)__shfl_xor((int)x, o, G);
    return x;
}
template <int G>
__device__ __forceinline__ uint32_t grp_sum(uint32_t x) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o, G);
    return x;
}
template <int G>
__device__ __forceinline__ void grp_argmin(double& key, int& idx) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) {
        const double ok = __shfl_xor(key, o, G);
        const int oi = __shfl_xor(idx, o, G);
        if (ok < key || (ok == key && oi < idx)) { key = ok; idx = oi; }
    }
}
struct PlanAcc {
    int lane_speed[NL];                     // the int-truncated lane speed where bit l of ls_set
    int ls_set;                             // (else P.max_speed)
    double next_s[NL];
    int open_m;                             // lane_open, bit l
    int in_id; double in_s;
    int t_id[NL];
    double t_s[NL];
    // iteration index of each running minimum, kItBits each: next_s[l] at field l, the target-lane
    // car of lane l at field NL + l, the in-lane car at field 2 NL (the follow cars' velocities are
    // re-read from that index after the pass)
    static constexpr int kItBits = 64 / (2 * NL + 1);
    static constexpr uint64_t kItMask = (1ull << kItBits) - 1;
    uint64_t its;
    int nmatched;
    __device__ __forceinline__ int it_of(int f) const { return (int)((its >> (kItBits * f)) & kItMask); }
    __device__ __forceinline__ void set_it(int f, int it) {
        its = (its & ~(kItMask << (kItBits * f))) | ((uint64_t)it << (kItBits * f));
    }
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int l = 0; l < NL; l++) {
            lane_speed[l] = 0; next_s[l] = 1000;
            t_id[l] = -1; t_s[l] = 0;
        }
        open_m = (1 << NL) - 1;
        ls_set = 0; in_id = -1; in_s = 0; its = 0; nmatched = 0;
    }
    // one matched car (iteration index it) with its Frenet state
    __device__ __forceinline__ void add(const pp_params& P, const EgoSt& e, int T_in, int it, int id,
                                        double cs, double cd, int clane, double cvs, double cvd) {
        const double ego_s = e.ego_s, ego_vs = e.ego_vs, dt0 = e.dt0;
        nmatched++;
        // planner (src/main.cpp:379-444)
        const double sp = cs + cvs * dt0;
        if (sp > ego_s) {
            // the first car (in iteration order) with the smallest sp sets next_s; lane_speed
            // comes from it if it is within 200 m (an earlier, larger minimum never is then)
            // (next_s == 1000: still the initial value, which no car can set, so it wins the tie)
            const double ns = sel(next_s, clane);
            if (sp < ns || (sp == ns && ns != 1000 && it < it_of(clane))) {
                put(next_s, clane, sp);
                set_it(clane, it);
                set_speed(P, ego_s, clane, sp, cvs);
            }
        }
        bool open = true;
        double add = 2;
        if (T_in == clane) add = 0;
        const double min_dist = P.car_length + P.safety_distance + add;
        if (fabs(ego_s - sp) < min_dist) open = false;
        if (sp > ego_s && cvs < ego_vs) {
            const double car_dist = sp - ego_s - P.car_length - P.safety_distance - add;
            const double sd = ego_vs - cvs;
            const double dtm = sd / P.relaxed_acc;
            const double ddist = ego_vs * dtm - sd / 2 * dtm;
            if (car_dist < ddist) open = false;
        }
        if (sp < ego_s && cvs > ego_vs && sp + 50 > ego_s) {
            const double car_dist = ego_s - sp - P.car_length - P.safety_distance - add;
            const double sd = cvs - ego_vs;
            double dtm = sd / P.relaxed_acc;
            if (T_in == e.ego_lane) dtm += 2;
            const double md = sd * dtm;
            if (car_dist < md) open = false;
        }
        if (!open) open_m &= ~(1 << clane);
        // follow cars (src/main.cpp:1391-1409); the target-lane choice for every candidate lane
        const double s0 = cs + cvs * dt0;
        const double d0 = cd + cvd * dt0;
        if (s0 > ego_s && fabs(d0 - e.ego_d) < 3) {
            if (in_id == -1 || in_s > s0 || (in_s == s0 && it < it_of(2 * NL))) {
                in_id = id; in_s = s0; set_it(2 * NL, it);
            }
        }
#pragma unroll
        for (int L = 0; L < NL; L++) {
            if (s0 >= ego_s - P.car_length - P.safety_distance && fabs(d0 - lane_offset(L)) < 3) {
                if (t_id[L] == -1 || t_s[L] > s0 || (t_s[L] == s0 && it < it_of(NL + L))) {
                    t_id[L] = id; t_s[L] = s0; set_it(NL + L, it);
                }
            }
        }
    }
    // the lane's speed where car (sp, cvs) holds next_s of its lane (src/main.cpp:385-399)
    __device__ __forceinline__ void set_speed(const pp_params& P, double ego_s, int l, double sp, double cvs) {
        if (sp - ego_s < 200) {
            int speed = (int)cvs;
            if (speed > P.max_speed) speed = (int)P.max_speed;
            if (sp - ego_s > 100)
                speed = (int)(speed + (P.max_speed - speed) * (sp - ego_s - 100) / (200.0 - 100.0));
            put(lane_speed, l, speed);
            ls_set |= 1 << l;
        } else {
            ls_set &= ~(1 << l);
        }
    }
    // G cars at once, one per lane of the group (car it = this lane's iteration index; valid: a
    // matched car), all with iteration indices above every car added before: the same state as
    // add() over them in iteration order. Every selection is a minimum of (key, iteration index),
    // reduced over the group by shuffles and merged into the running one by add()'s own rule; the
    // per-car terms (planner keys, lane_open) are computed by each lane for its own car. The
    // caller keeps add() for groups holding a car whose id is the 'no car' sentinel -1, which
    // add() lets any later car replace.
    template <int G>
    __device__ __forceinline__ void add_group(const pp_params& P, const EgoSt& e, int T_in, bool valid, int it,
                                              int id, double cs, double cd, int clane, double cvs, double cvd) {
        const double ego_s = e.ego_s, ego_vs = e.ego_vs, dt0 = e.dt0;
        const double kInf = __builtin_inf();
        constexpr int kNone = 0x7fffffff;
        nmatched += (int)grp_sum<G>(valid ? 1u : 0u);
        const double sp = cs + cvs * dt0;
        // next_s per lane: the first car with the smallest sp in (ego_s, 1000)
#pragma unroll
        for (int l = 0; l < NL; l++) {
            double k = valid && clane == l && sp > ego_s && sp < 1000 ? sp : kInf;
            int ki = k == kInf ? kNone : it;
            grp_argmin<G>(k, ki);
            const double wcvs = __shfl(cvs, ki == kNone ? 0 : ki - (it - (int)(threadIdx.x % G)), G);
            const double ns = sel(next_s, l);
            if (ki != kNone && (k < ns || (k == ns && ns != 1000 && ki < it_of(l)))) {
                put(next_s, l, k);
                set_it(l, ki);
                set_speed(P, ego_s, l, k, wcvs);
            }
        }
        // lane_open (src/main.cpp:401-444): a lane closes if any of its cars closes it
        bool open = true;
        {
            double add = 2;
            if (T_in == clane) add = 0;
            const double min_dist = P.car_length + P.safety_distance + add;
            if (fabs(ego_s - sp) < min_dist) open = false;
            if (sp > ego_s && cvs < ego_vs) {
                const double car_dist = sp - ego_s - P.car_length - P.safety_distance - add;
                const double sd = ego_vs - cvs;
                const double dtm = sd / P.relaxed_acc;
                const double ddist = ego_vs * dtm - sd / 2 * dtm;
                if (car_dist < ddist) open = false;
            }
            if (sp < ego_s && cvs > ego_vs && sp + 50 > ego_s) {
                const double car_dist = ego_s - sp - P.car_length - P.safety_distance - add;
                const double sd = cvs - ego_vs;
                double dtm = sd / P.relaxed_acc;
                if (T_in == e.ego_lane) dtm += 2;
                const double md = sd * dtm;
                if (car_dist < md) open = false;
            }
        }
        open_m &= ~(int)grp_or<G>(valid && !open ? 1u << clane : 0u);
        // follow cars (src/main.cpp:1391-1409): the in-lane car, the target-lane car of each lane
        const double s0 = cs + cvs * dt0;
        const double d0 = cd + cvd * dt0;
        const int r0 = (int)(threadIdx.x % G), itb = it - r0;    // the group's first iteration index
        {
            double k = valid && s0 > ego_s && fabs(d0 - e.ego_d) < 3 ? s0 : kInf;
            int ki = valid && s0 > ego_s && fabs(d0 - e.ego_d) < 3 ? it : kNone;
            grp_argmin<G>(k, ki);
            const int wid = __shfl(id, ki == kNone ? 0 : ki - itb, G);
            if (ki != kNone && (in_id == -1 || in_s > k || (in_s == k && ki < it_of(2 * NL)))) {
                in_id = wid; in_s = k; set_it(2 * NL, ki);
            }
        }
#pragma unroll
        for (int L = 0; L < NL; L++) {
            const bool q = valid && s0 >= ego_s - P.car_length - P.safety_distance && fabs(d0 - lane_offset(L)) < 3;
            double k = q ? s0 : kInf;
            int ki = q ? it : kNone;
            grp_argmin<G>(k, ki);
            const int wid = __shfl(id, ki == kNone ? 0 : ki - itb, G);
            if (ki != kNone && (t_id[L] == -1 || t_s[L] > k || (t_s[L] == k && ki < it_of(NL + L)))) {
                t_id[L] = wid; t_s[L] = k; set_it(NL + L, ki);
            }
        }
    }
};


// TrajectoryBuilder::build start pose (src/main.cpp:583-610): the last kept previous point and the
// heading of the last kept step, or the ego pose
__device__ __forceinline__ void start_pose(const pp_scene_batch& in, int64_t S, int64_t s, const EgoSt& e,
                                           double& pos_x, double& pos_y, double& angle) {
    if (e.K == 0) {
        pos_x = e.ego_x; pos_y = e.ego_y;
        angle = e.yaw * kPi / 180;
    } else {
        pos_x = in.prev_x[9 * S + s]; pos_y = in.prev_y[9 * S + s];
        const double vx = pos_x - e.p8x, vy = pos_y - e.p8y;
        if (vx * vx + vy * vy < kEps) angle = e.yaw * kPi / 180;
        else angle = ppg::atan2(pos_y - e.p8y, pos_x - e.p8x);       // glibc's atan2, bit for bit
    }
}
// The frame's rotations tv = cos(-a), sin(-a), cos(a), sin(a) as the reference's libm computes
// them. glibc's sin is odd and its cos even bit for bit (both reduce |x| and apply the sign last;
// tests/test_glibcm.py checks the restatement on 3.9 M arguments), so two evaluations give all
// four: cos(-a) = cos(a), sin(-a) = -sin(a). G > 1: lane r of the group computes tv[r] (r < 4;
// the others hold nothing), except when the restated reduction fails (every lane then holds all
// four, from the library's own reduction)
template <int G>
__device__ __forceinline__ void frame_trig(double angle, int r, double tv[4]) {
    bool tfail = false;
    if (G == 1) {
        tfail = !ppg::cos(angle, tv[2]);
        tfail |= !ppg::sin(angle, tv[3]);
        tv[0] = tv[2];
        tv[1] = -tv[3];
    } else {
#pragma unroll
        for (int t = 0; t < 4; t++) {
            if (t % G != r) continue;
            double v;
            tfail |= !((t & 1) ? ppg::sin(angle, v) : ppg::cos(angle, v));
            tv[t] = t == 1 ? -v : v;
        }
    }
    if (G > 1) tfail = grp_or<G>(tfail ? 1u : 0u) != 0u;
    if (tfail) {                              // every lane: both pairs (rare)
        double sm, cm, sp, cp;
        ppm::sincos_pp<true>(-angle, sm, cm);
        ppm::sincos_pp<true>(angle, sp, cp);
        tv[0] = cm; tv[1] = sm; tv[2] = cp; tv[3] = sp;
    }
}

// The rest of K1 after the car pass (src/main.cpp:447-484, 1358-1438, 583-610, 786-823): scores
// and the target lane, LimitSpeed for the in-lane car (task 0) and each lane's target car (task
// 1 + L), k_cand<false>'s range checks, the build start pose and the frame rotations (tasks 0-3:
// cos(-a), sin(-a), cos(a), sin(a)). G > 1: the tasks are spread over the lanes of the group
// (lane r takes tasks r, r + G, ...) and lane 0 writes the scene's record.
template <int G>
__device__ __forceinline__ void prep_finish(const pp_scene_batch& in, const pp_params& P, const PrepV& pv,
                                            pp_scene_info* info, uint32_t* out_status, const GroupBits& gb,
                                            int64_t S, int64_t Sv, int64_t s, int64_t v, int draw, bool tab,
                                            int r, int T_in, const EgoSt& e, const PlanAcc& a,
                                            uint32_t status) {
    // scores + argmax (src/main.cpp:447-484)
    int best_lane = e.ego_lane;
    double best_score = 0;
    double score[NL];
#pragma unroll
    for (int lane = 0; lane < NL; lane++) {
        score[lane] = 0;
        if (lane != e.ego_lane && !((a.open_m >> lane) & 1)) continue;
        const double lsp = ((a.ls_set >> lane) & 1) ? (double)a.lane_speed[lane] : P.max_speed;
        const double speed_score = s_min(lsp / P.max_speed, 1.0);
        const double distance_score = 1 - fabs((double)(T_in - lane)) / 2;
        const double free_score = s_min(1.0, a.next_s[lane] / 100);
        const double total = speed_score + distance_score / 2 + free_score;
        score[lane] = total;
        if (total > best_score) { best_score = total; best_lane = lane; }
    }
    int T;
    if (abs(e.ego_lane - best_lane) > 1) {
        const int nl = best_lane > e.ego_lane ? e.ego_lane + 1 : e.ego_lane - 1;
        T = ((a.open_m >> nl) & 1) ? nl : e.ego_lane;
        status |= PP_ST_JUMP_RULE;
    } else {
        T = best_lane;
    }
    const int open_mask = a.open_m;
    if (open_mask != (1 << NL) - 1) status |= PP_ST_LANE_CLOSED;
    if (T != e.ego_lane) {                                             // src/main.cpp:1358-1369
        const double dtl = lane_offset(T);
        const double diff = fabs(e.ego_vd * 1.0 + e.ego_d - dtl);
        if (diff > 6.0) { T = e.ego_lane; status |= PP_ST_TOO_FAR; }
    }
    // LimitSpeed for the in-lane car and the per-lane target car (src/main.cpp:1411-1438); the
    // reference's "no car" is id -1 (:1383-1432): a chosen car whose id is -1 reads as none; ids
    // are what :1411 compares. k_cand<false> divides by reciprocals without range checks: every
    // speed and ramp time of the scene must be in range (else kLimSlow)
    int lim_mask = 0;
    bool ok = true;
    for (int t = r; t < 1 + NL; t += G) {
        bool has = a.in_id != -1, in_lane = true;
        double fs = a.in_s;
        int fit = a.it_of(2 * NL);
#pragma unroll
        for (int L = 0; L < NL; L++)
            if (t == 1 + L) { has = a.t_id[L] != -1 && a.t_id[L] != a.in_id; in_lane = false; fs = a.t_s[L]; fit = a.it_of(NL + L); }
        if (!has) continue;
        double ts, tt, fvx, fvy;
        bool col;
        car_velocity(in, P, S, s, draw, tab, fit, fvx, fvy);
#ifdef PP_ABL_NOLIM
        ts = fs; tt = fvx; col = false; const int code = 0;   // (ablation build: wrong results)
#else
        const int code = limit_speed(P, fvx, fvy, fs, e.ego_s, e.ego_speed, e.ego_acc, in_lane, ts, tt, col);
#endif
        status |= limit_flag(code) | (col ? PP_ST_COLLISION : 0u);
        if (t == 0) { pv.in_ts[v] = ts; pv.in_tt[v] = tt; }
        else { pv.l_ts[(t - 1) * Sv + v] = ts; pv.l_tt[(t - 1) * Sv + v] = tt; }
        lim_mask |= 1 << t;
        ok = ok && speed_in_range(ts) && speed_in_range(tt);
    }
    for (int k = r; k < P.n_speeds; k += G) {
        const double vk = cand_speed(P, e.ego_speed, k);
        ok = ok && speed_in_range(vk) && speed_in_range(fabs(e.ego_speed - vk) / P.relaxed_acc);
    }
    ok = ok && speed_in_range(e.ego_speed);
    if (G > 1) {
        status = grp_or<G>(status);
        lim_mask = (int)grp_or<G>((uint32_t)lim_mask);
        ok = grp_or<G>(ok ? 0u : 1u) == 0u;
    }
    // TrajectoryBuilder::build start pose (src/main.cpp:583-610) + frame rotations (:786-823)
    // (gb.pose_by_wave: the wave step's phase-A waves compute and record the start pose, its
    // rotations and the heading's kLimSlow bit themselves, off K1's critical path)
    double pos_x = 0, pos_y = 0, angle = 0;
    if (!gb.pose_by_wave) {
        start_pose(in, S, s, e, pos_x, pos_y, angle);
        // heading beyond the hot loop's medium trig range (only from an absurd telemetry yaw): the
        // scene is evaluated by the k_cand<true> instantiation with the library's large reduction
        if (!(fabs(angle) <= kSlowAngle)) lim_mask |= kLimSlow;
    }
    if (!ok) lim_mask |= kLimSlow;
    if ((lim_mask & kLimSlow) && r == 0 && gb.bits) {   // (k_step_small: no bitmap)
        const int64_t g0 = gb.BPS == 1 ? s / gb.SPB : gb.BPS < 0 ? s * gb.C / 256 : s * gb.BPS;
        const int nb = gb.BPS < 0 ? (int)(((s + 1) * gb.C - 1) / 256 - g0 + 1) : gb.BPS;
        for (int b = 0; b < nb; b++) {
            const uint32_t bit = 1u << ((g0 + b) & 31);
            const uint32_t old = atomicOr(&gb.bits[(g0 + b) >> 5], bit);
            if (!(old & bit) && gb.list) gb.list[atomicAdd(gb.count, 1u)] = (uint32_t)(g0 + b);
        }
    }
    // the frame's rotations cos(-angle), sin(-angle) (:786-787) and cos(angle), sin(angle)
    // (:822-823) as the reference's libm computes them (pp_glibcm.h): every knot is a product with
    // them, so the spline and every path position carry their exact bits. Headings of 1e8 rad and
    // more (only from an absurd telemetry yaw) are outside the restated reduction.
    if (!gb.pose_by_wave) {
        double tv[4];
#ifdef PP_ABL_NOTRIG
        tv[0] = tv[2] = angle; tv[1] = tv[3] = -angle;           // (ablation build: wrong results)
#else
        frame_trig<G>(angle, r, tv);
#endif
        double* const tdst[4] = {pv.ca_m, pv.sa_m, pv.ca_p, pv.sa_p};
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (G == 1 || t % G == r) tdst[t][v] = tv[t];
        if (r == 0) { pv.pos_x[v] = pos_x; pv.pos_y[v] = pos_y; pv.angle[v] = angle; }
    }
    if (r != 0) return;
    pv.ego_speed[v] = e.ego_speed; pv.ego_d[v] = e.ego_d; pv.ego_vd[v] = e.ego_vd;
#pragma unroll
    for (int l = 0; l < NL; l++) { pv.ratio[l * Sv + v] = e.ratio[l]; pv.score[l * Sv + v] = score[l]; }
    pv.K[v] = e.K; pv.ref_wp[v] = e.ref_wp; pv.T[v] = T; pv.ego_lane[v] = e.ego_lane;
    pv.open_mask[v] = open_mask; pv.lim_mask[v] = lim_mask; pv.status[v] = status;
    if (draw == 0) out_status[s] = 0;        // k_cand ORs its flags in (atomics when a scene spans blocks)
    if (info && draw == 0) {
        pp_scene_info I = {};
        I.ego_x = e.ego_x; I.ego_y = e.ego_y; I.ego_speed = e.ego_speed; I.ego_acc = e.ego_acc;
        I.ego_s = e.ego_s; I.ego_d = e.ego_d; I.ego_vs = e.ego_vs; I.ego_vd = e.ego_vd;
        for (int l = 0; l < NL; l++) { I.ref_ratio[l] = e.ratio[l]; I.lane_score[l] = score[l]; }
        I.ref_wp = e.ref_wp; I.ego_lane = e.ego_lane; I.target_lane = T; I.lane_open_mask = open_mask;
        I.n_matched_cars = a.nmatched; I.in_lane_car = a.in_id;
        info[s] = I;
    }
}

// Monte-Carlo sensor noise on one car row (include/pp.h pp_params)
__device__ __forceinline__ void car_noise(const pp_params& P, int64_t s, int draw, int row, double& cx,
                                          double& cy, double& cvx, double& cvy) {
    const uint64_t gs = (uint64_t)(P.noise_first_scene + s);
    double g[4];
#ifndef PP_G4
#define PP_G4 1
#endif
    if (PP_G4) ppsynth::mc_gauss4(P.noise_seed, gs, draw, row, g);      // (mc_gauss q = 0..3)
    else for (int q = 0; q < 4; q++) g[q] = ppsynth::mc_gauss(P.noise_seed, gs, draw, row, q);
    cx += P.noise_pos_sigma * g[0];
    cy += P.noise_pos_sigma * g[1];
    cvx += P.noise_vel_sigma * g[2];
    cvy += P.noise_vel_sigma * g[3];
}

// kW4: the 4-waves-per-SIMD instantiation (<= 128 VGPRs): for batches whose wave count fills
// whole rounds of 4 waves per SIMD better than of 3 (prep_w4 in pp_eval)
#ifndef PP_SORT_DMAX
#define PP_SORT_DMAX 16          // k_prep sorts a scene's rows nearest first below this many draws
#endif
#ifndef PP_SORT_K0
#define PP_SORT_K0 0             // 1: k_sort_cars by default (PP_DBG_SORT_CARS switches it per call)
#endif
// K0 (round 6, PP_SORT_K0): each scene's cars in k_prep's visiting order, visit-major.
// k_prep visits a scene's rows nearest first (below), and read them in that order straight from the
// batch's row-major arrays: a wave's load of visit k gathers 64 scenes' rows from up to 12 rows,
// each cache line partly used and fetched again at later visits (FETCH ~7x the scene record,
// DESIGN.md §4). k_sort_cars computes the same order (the same keys, the same network, the same
// identity-order rules) and writes the rows permuted into visit-major arrays x[k][s], ... through a
// per-lane LDS column, so k_prep's visit k reads 64 consecutive values per field. Only for batches
// without a car table, fewer than PP_SORT_DMAX draws and at most 16 rows per scene (the host's
// condition); the values are copies, so k_prep's results are the same bits.
struct SortedCars {
    double *x, *y, *vx, *vy;      // [k][S], k < rows: the k-th visited row's fields
    int* id;                      // [k][S]
    uint64_t* order;              // [S]: the visiting order, one row index per nibble
    int rows;                     // min(car_stride, 16); 0: not in use
};
__device__ __forceinline__ uint64_t car_order(const pp_scene_batch& in, int64_t S, int64_t s, double ex,
                                              double ey, int iters) {
    uint64_t order = 0xFEDCBA9876543210ull;
    if (!(iters > 1 && iters <= 16)) return order;
    uint32_t key[16];
    bool neg = false;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        key[j] = 0xFFFFFFF0u | (uint32_t)j;
        if (j < iters) {
            const int64_t ix = (int64_t)j * S + s;
            const double dx = in.car_x[ix] - ex, dy = in.car_y[ix] - ey;
            const float f = (float)(dx * dx + dy * dy);
            key[j] = (__float_as_uint(f) & ~15u) | (uint32_t)j;
            neg |= in.car_id[ix] < 0;
        }
    }
#pragma unroll
    for (int pw = 1; pw < 16; pw <<= 1)
#pragma unroll
        for (int k = pw; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % pw; j < 16 - k; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; i++)
                    if ((i + j) / (2 * pw) == (i + j + k) / (2 * pw)) {
                        const uint32_t lo = key[i + j] < key[i + j + k] ? key[i + j] : key[i + j + k];
                        const uint32_t hi = key[i + j] < key[i + j + k] ? key[i + j + k] : key[i + j];
                        key[i + j] = lo; key[i + j + k] = hi;
                    }
    if (neg) return order;
    order = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) order |= (uint64_t)(key[j] & 15u) << (4 * j);
    return order;
}
__global__ __launch_bounds__(256) void k_sort_cars(pp_scene_batch in, SortedCars sc, int64_t s0, int64_t s1) {
    __shared__ double col[16 * 256];          // this lane's rows of one field: col[j * 256 + lane]
    const int64_t S = in.n_scenes;
    const int t = threadIdx.x;
    const int64_t s = s0 + (int64_t)blockIdx.x * 256 + t;
    if (s >= s1) return;                      // (no barrier below: every lane uses its own column)
    int iters = in.n_cars[s];
    if (iters > in.car_stride) iters = in.car_stride;
    // the ego position k_prep's keys use (prep_ego: the last kept point when 10 are kept)
    const int np = in.n_prev[s];
    const double ex = np >= PP_PREV_KEEP ? in.prev_x[9 * S + s] : in.ego_x[s];
    const double ey = np >= PP_PREV_KEEP ? in.prev_y[9 * S + s] : in.ego_y[s];
    const uint64_t order = car_order(in, S, s, ex, ey, iters);
    sc.order[s] = order;
    const double* src[4] = {in.car_x, in.car_y, in.car_vx, in.car_vy};
    double* dst[4] = {sc.x, sc.y, sc.vx, sc.vy};
#pragma unroll
    for (int f = 0; f < 4; f++) {
        for (int j = 0; j < iters; j++) col[j * 256 + t] = src[f][(int64_t)j * S + s];
        for (int k = 0; k < iters; k++) dst[f][(int64_t)k * S + s] = col[(int)((order >> (4 * k)) & 15) * 256 + t];
    }
    // the ids in the low half of this lane's own double slots (the waves of the block run without a
    // barrier: a lane must never touch another lane's slots)
    int* icol = (int*)col;
    for (int j = 0; j < iters; j++) icol[2 * (j * 256 + t)] = in.car_id[(int64_t)j * S + s];
    for (int k = 0; k < iters; k++) sc.id[(int64_t)k * S + s] = icol[2 * ((int)((order >> (4 * k)) & 15) * 256 + t)];
}

// kK0: k_sort_cars ran (srt holds the rows visit-major); a separate instantiation, so the default
// path carries no test of it
template <bool kLdsMap, bool kW4 = false, bool kK0 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kW4 ? 4 : kPrepWaves))) void k_prep(MapG mg, pp_scene_batch in, pp_params P, PrepV pv,
                                              pp_scene_info* info, uint32_t* out_status, GroupBits gb,
                                              int64_t v0, int64_t v1, SortedCars srt) {
    extern __shared__ __attribute__((aligned(16))) double smap[];
    const int n = mg.n;
#ifdef PP_TRACE
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)(kTraceMax - kTraceK1)) {
        trace_at(kTraceK1 + blockIdx.x, 0);
        g_trace[8 * (kTraceK1 + blockIdx.x) + 7] = trace_hwid();
    }
#endif
    // the approach table: in LDS after the map (16-B aligned) in k_prep<true, false> (the host
    // sizes the launch for it, or passes none), else in global memory
#ifndef PP_ATAB_LDS
#define PP_ATAB_LDS 1
#endif
    constexpr bool kAtabL = kLdsMap && !kW4 && PP_ATAB_LDS;
    double* satab = smap + ((kMapArrays * n + 1) & ~1);
    if (kLdsMap) {
        stage_map(smap, mg.buf, kMapArrays * n);
        if (kAtabL && mg.atab) stage_map(satab, mg.atab, kAtabD * n);
        __syncthreads();
    }
#ifdef PP_TRACE
    if (threadIdx.x == 0 && blockIdx.x < (unsigned)(kTraceMax - kTraceK1)) trace_at(kTraceK1 + blockIdx.x, 1);
#endif
    MapV m = map_view(kLdsMap ? smap : mg.buf, n, mg.fastm);
    m.wg = mg.wg;                         // the closest-waypoint cell table (global memory)
    m.wseg = mg.wseg;                     // reference segment lengths and reciprocals (global memory)
    m.atab = kAtabL ? satab : mg.atab;    // the approach table (LDS or global memory)
    m.atab_on = mg.atab != nullptr;
    // one lane per evaluation v = s * D + d (scene s, Monte-Carlo draw d; D = 1 without noise):
    // inputs are read at scene s (stride S), the prep record is written at v (stride Sv)
    const int64_t S = in.n_scenes;
    const int D = P.n_draws > 1 ? P.n_draws : 1;
    const int64_t Sv = S * D;
    // evaluations [v0, v1) of the batch (pp_eval's chunked pipeline launches K1 per chunk)
    const int64_t v = v0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= v1 || v >= Sv) return;
    const int64_t s = D == 1 ? v : v / D;
    const int draw = (int)(v - s * D);

    EgoSt e;
    PP_REGION_K("ego");
    prep_ego<1>(m, in, P, S, s, 0, e);
    PP_REGION_K("sort");
    uint32_t status = e.status;
    const int T_in = in.prev_target_lane[s];
    PlanAcc a;
    a.init();
    int ncar = in.n_cars[s];
    if (ncar > in.car_stride) ncar = in.car_stride;
    // Without a car table: the frame's rows in order (ascending ids). With one (the reference's
    // persistent std::map): its tab_slots slots in order (ascending ids, include/pp.h), each car
    // either reported this frame (re-matched; slot overwritten, or erased when matching fails,
    // src/main.cpp:1329-1348) or taken from its stale slot.
    const bool tab = in.tab_valid != nullptr;
#ifdef PP_ABL_NOCARS
    const int iters = 0;                    // (ablation build: wrong results)
#else
    const int iters = tab ? in.tab_slots : ncar;
#endif
    // Visiting order (PlanAcc: any order once ties compare the iteration index). Without a car
    // table the rows are visited nearest first (squared distance to the ego, a 4-bit row index in
    // the low mantissa bits of a float key, sorted by a Batcher network): the k-th visit of every
    // lane of a wave then walks a similar number of lane segments in lane_matching, which is where
    // the divergence was. With a table, or a negative car id (the reference's -1 'no car'
    // sentinel), the identity order is kept. (more than 16 rows: the identity order.) So do
    // Monte-Carlo batches of 16 draws or more: a wave's lanes are the draws of at most 4 scenes
    // (v = s D + d), which visit the same rows in lockstep anyway
    uint64_t order = 0xFEDCBA9876543210ull;
    bool sorted = false;
    // K0 ran (k_sort_cars): its order, and the rows in visit-major arrays
    constexpr bool k0 = kK0;
    if (k0) { order = srt.order[s]; sorted = true; }
#ifdef PP_ABL_NOSORT
    if (false) {
#else
    if (!k0 && !tab && iters > 1 && iters <= 16 && D < PP_SORT_DMAX) {
#endif
        uint32_t key[16];
        bool neg = false;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            key[j] = 0xFFFFFFF0u | (uint32_t)j;
            if (j < iters) {
                const int64_t ix = (int64_t)j * S + s;
                const double dx = in.car_x[ix] - e.ego_x, dy = in.car_y[ix] - e.ego_y;
                const float f = (float)(dx * dx + dy * dy);
                key[j] = (__float_as_uint(f) & ~15u) | (uint32_t)j;
                neg |= in.car_id[ix] < 0;
            }
        }
#pragma unroll
        for (int pw = 1; pw < 16; pw <<= 1)
#pragma unroll
            for (int k = pw; k >= 1; k >>= 1)
#pragma unroll
                for (int j = k % pw; j < 16 - k; j += 2 * k)
#pragma unroll
                    for (int i = 0; i < k; i++)
                        if ((i + j) / (2 * pw) == (i + j + k) / (2 * pw)) {
                            const uint32_t lo = key[i + j] < key[i + j + k] ? key[i + j] : key[i + j + k];
                            const uint32_t hi = key[i + j] < key[i + j + k] ? key[i + j + k] : key[i + j];
                            key[i + j] = lo; key[i + j + k] = hi;
                        }
        if (!neg) {
            order = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) order |= (uint64_t)(key[j] & 15u) << (4 * j);
            sorted = true;
        }
    }
    static_assert(PP_MAX_CARS <= (1 << PlanAcc::kItBits), "iteration index fields");
    int p = 0;                              // next unread row (table mode)
    for (int kk = 0; kk < iters; kk++) {
        PP_REGION_K("carload");
        const int it = sorted ? (int)((order >> (4 * kk)) & 15) : kk;
        int row = it;
        const int64_t tix = (int64_t)it * S + s;
        // table mode: slot `it` holds car id sid (slots in ascending id order, include/pp.h)
        const int sid = tab ? (in.tab_id ? in.tab_id[tix] : it) : 0;
        if (tab) {
            while (p < ncar && in.car_id[(int64_t)p * S + s] < sid) p++;    // ids must ascend
            row = (p < ncar && in.car_id[(int64_t)p * S + s] == sid) ? p++ : -1;
        }
        int id;
        double cx, cy, cvx, cvy, cs, cd, cvs, cvd;
        int clane = 0;
        if (row >= 0) {
            if (k0) {                       // visit kk's row, visit-major (coalesced)
                const int64_t kx = (int64_t)kk * S + s;
                id = srt.id[kx];
                cx = srt.x[kx]; cy = srt.y[kx]; cvx = srt.vx[kx]; cvy = srt.vy[kx];
            } else {
                const int64_t ix = (int64_t)row * S + s;
                id = in.car_id[ix];
                cx = in.car_x[ix]; cy = in.car_y[ix]; cvx = in.car_vx[ix]; cvy = in.car_vy[ix];
            }
            if (draw > 0) car_noise(P, s, draw, row, cx, cy, cvx, cvy);
            int nwp = 0;
            PP_DIAGC(17, true);
            PP_REGION_K("match");
            if (!lane_match(m, e.ref_wp, e.ratio, cx, cy, cs, cd, clane, nwp)) {
                status |= PP_ST_CAR_UNMATCHED;
                if (tab) in.tab_valid[tix] = 0;
                continue;
            }
            PP_REGION_K("proj");
#ifdef PP_ABL_NOPROJ
            cvs = cvx; cvd = cvy;                                 // (ablation build: wrong results)
#else
            project_speed(m, cvx, cvy, nwp, cvs, cvd);
#endif
            if (tab) {
                in.tab_valid[tix] = 1; in.tab_lane[tix] = clane;
                in.tab_s[tix] = cs; in.tab_d[tix] = cd; in.tab_vs[tix] = cvs; in.tab_vd[tix] = cvd;
                in.tab_vx[tix] = cvx; in.tab_vy[tix] = cvy;
            }
        } else {
            if (!in.tab_valid[tix]) continue;
            id = sid;
            clane = in.tab_lane[tix];
            cs = in.tab_s[tix]; cd = in.tab_d[tix]; cvs = in.tab_vs[tix]; cvd = in.tab_vd[tix];
        }
        PP_REGION_K("plan");
#ifdef PP_ABL_NOPLAN
        a.nmatched += id + clane; a.in_s += cs + cd + cvs + cvd;  // (ablation build: wrong results)
#else
        a.add(P, e, T_in, it, id, cs, cd, clane, cvs, cvd);
#endif
    }
    PP_REGION_K("finish");
    prep_finish<1>(in, P, pv, info, out_status, gb, S, Sv, s, v, draw, tab, 0, T_in, e, a, status);
#ifdef PP_TRACE
    if ((threadIdx.x & 63) == 0 && blockIdx.x < (unsigned)(kTraceMax - kTraceK1))
        trace_at(kTraceK1 + blockIdx.x, 2 + (threadIdx.x >> 6));
#endif
}

// K1 for small batches: a group of G lanes per evaluation (G = 2 ... 16; kernels k_prep_g2 ... k_prep_g16), so that a batch of a few
// thousand scenes still fills the chip (BASELINE config 2: 4,096 scenes). Lane r of a group matches
// rows r, r + G, ... (coalesced across the group) and scans every G-th waypoint for the Frenet
// frame; the planner's pass then runs over each round's G cars in ascending row order on every
// lane of the group (the cars' Frenet states exchanged by lane shuffles), i.e. in the reference's
// own iteration order. No car table (pp_eval picks k_prep for table mode).
template <int G>
__device__ __forceinline__ void prep_grp_eval(const MapV& m, const pp_scene_batch& in, const pp_params& P,
                                              const PrepV& pv, pp_scene_info* info, uint32_t* out_status,
                                              const GroupBits& gb, int64_t v, int r);
template <bool kLdsMap, int G>
__device__ __forceinline__ void prep_grp_body(MapG mg, pp_scene_batch in, pp_params P, PrepV pv,
                                              pp_scene_info* info, uint32_t* out_status, GroupBits gb) {
    static_assert(G >= 2 && G <= 16 && (G & (G - 1)) == 0, "group: a power of two in [2, 16]");
    extern __shared__ __attribute__((aligned(16))) double smap[];
    const int n = mg.n;
    if (kLdsMap) {
        stage_map(smap, mg.buf, kMapArrays * n);
        __syncthreads();
    }
    const MapV m = map_view(kLdsMap ? smap : mg.buf, n, mg.fastm);
    const int64_t Sv = in.n_scenes * (P.n_draws > 1 ? P.n_draws : 1);
    const int r = (int)(threadIdx.x % G);
    const int64_t v = (int64_t)blockIdx.x * (blockDim.x / G) + threadIdx.x / G;
    if (v >= Sv) return;                      // whole groups leave together
    prep_grp_eval<G>(m, in, P, pv, info, out_status, gb, v, r);
}

// the grouped K1's planner pass: the group's cars at once (PlanAcc::add_group), or one at a time
#ifndef PP_GROUP_PASS
#define PP_GROUP_PASS 1
#endif
constexpr bool kGroupPass = PP_GROUP_PASS != 0;
// One evaluation v by the G lanes of a group (this one is lane r); every lane of the group runs it
template <int G>
__device__ __forceinline__ void prep_grp_eval(const MapV& m, const pp_scene_batch& in, const pp_params& P,
                                              const PrepV& pv, pp_scene_info* info, uint32_t* out_status,
                                              const GroupBits& gb, int64_t v, int r) {
    const int64_t S = in.n_scenes;
    const int D = P.n_draws > 1 ? P.n_draws : 1;
    const int64_t Sv = S * D;
    const int64_t s = D == 1 ? v : v / D;
    const int draw = (int)(v - s * D);

    EgoSt e;
    PP_TRACE_K1(0);
    prep_ego<G>(m, in, P, S, s, r, e);
    PP_TRACE_K1(1);
    uint32_t status = e.status;
    const int T_in = in.prev_target_lane[s];
    PlanAcc a;
    a.init();
    // row r of the first G rows, loaded with n_cars rather than after it (rows below car_stride
    // exist; the frame's K1 waits for one memory round trip here, not two)
    int pid0 = 0;
    double px0 = 0, py0 = 0, pvx0 = 0, pvy0 = 0;
    if (r < in.car_stride) {
        const int64_t ix = (int64_t)r * S + s;
        pid0 = in.car_id[ix];
        px0 = in.car_x[ix]; py0 = in.car_y[ix]; pvx0 = in.car_vx[ix]; pvy0 = in.car_vy[ix];
    }
    int ncar = in.n_cars[s];
    if (ncar > in.car_stride) ncar = in.car_stride;
    // Without a car table: the frame's rows. With one (the reference's persistent std::map, as
    // k_prep): its tab_slots slots in order, each either reported this frame (re-matched; the slot
    // overwritten, or erased when matching fails, src/main.cpp:1329-1348) or taken from its stale
    // slot. Iteration index = row or slot, as in k_prep.
    const bool tab = in.tab_valid != nullptr;
    const int iters = tab ? in.tab_slots : ncar;
    uint32_t ust = 0;
    for (int j0 = 0; j0 < iters; j0 += G) {
        const int j = j0 + r;
        int okl = 0, id = 0;                  // okl: matched | lane << 1
        double cs = 0, cd = 0, cvs = 0, cvd = 0;
        // table mode: slot j holds id sid; its reported row, if any (rows ascend by id: the first
        // row with that id, the row k_prep's merge pointer reaches). Slot ids ascend strictly; a
        // slot repeating its predecessor's id is padding (pp_cartable.h pads with INT32_MAX, which
        // may also be a real car's id): it matches no row, as k_prep's merge pointer has already
        // passed that row. The group's lanes load the rows' ids (row p0 + q in lane q) and every
        // lane scans them by shuffles: one round trip to memory for the ids, not one per row
        // visited (the single-frame kernel waits for every one of those).
        int trow = -1, sid = 0;
        // (frames of at most G rows: the rows' cars come along with their ids, and the found row's
        // by a shuffle; the slot's stored state is read with its id: no load waits on the search)
        double fx = 0, fy = 0, fvx = 0, fvy = 0;
        bool fgot = false;
        int sv = 0, sln = 0;
        double ss = 0, sd = 0, svs = 0, svd = 0;
        if (tab) {
            const bool live = j < iters;
            const int64_t tix = (int64_t)j * S + s;
            sid = live ? (in.tab_id ? in.tab_id[tix] : j) : 0;
            if (live) {
                sv = in.tab_valid[tix]; sln = in.tab_lane[tix];
                ss = in.tab_s[tix]; sd = in.tab_d[tix]; svs = in.tab_vs[tix]; svd = in.tab_vd[tix];
            }
            bool done = !live || (in.tab_id && j > 0 && in.tab_id[tix - S] >= sid);
            for (int p0 = 0; p0 < ncar; p0 += G) {
                const int pl = p0 + r;
                int pid = 0;
                double px = 0, py = 0, pvx = 0, pvy = 0;
                if (p0 == 0) {                // (the rows loaded ahead)
                    if (pl < ncar) { pid = pid0; px = px0; py = py0; pvx = pvx0; pvy = pvy0; }
                } else if (pl < ncar) {
                    const int64_t ix = (int64_t)pl * S + s;
                    pid = in.car_id[ix];
                }
                const int nq = ncar - p0 < G ? ncar - p0 : G;
                for (int q = 0; q < nq; q++) {
                    const int cid = __shfl(pid, q, G);
                    if (!done && cid >= sid) { if (cid == sid) trow = p0 + q; done = true; }
                }
                if (ncar <= G) {              // (group-uniform)
                    const int src = trow >= 0 ? trow : 0;
                    fx = __shfl(px, src, G); fy = __shfl(py, src, G);
                    fvx = __shfl(pvx, src, G); fvy = __shfl(pvy, src, G);
                    fgot = trow >= 0;
                }
                if (grp_or<G>(done ? 0u : 1u) == 0u) break;
            }
        }
        PP_TRACE_K1(2);
        if (j < iters) {
            const int64_t tix = (int64_t)j * S + s;
            int row = j;
            if (tab) { row = trow; id = sid; }
            if (row >= 0) {
                const int64_t ix = (int64_t)row * S + s;
                double cx, cy, cvx, cvy;
                if (fgot) {                   // (tab: the row's id is the slot's)
                    cx = fx; cy = fy; cvx = fvx; cvy = fvy;
                } else if (!tab && j0 == 0) { // row j = r: loaded ahead
                    id = pid0;
                    cx = px0; cy = py0; cvx = pvx0; cvy = pvy0;
                } else {
                    id = in.car_id[ix];
                    cx = in.car_x[ix]; cy = in.car_y[ix]; cvx = in.car_vx[ix]; cvy = in.car_vy[ix];
                }
                if (draw > 0) car_noise(P, s, draw, row, cx, cy, cvx, cvy);
                int nwp = 0, clane = 0;
                if (lane_match(m, e.ref_wp, e.ratio, cx, cy, cs, cd, clane, nwp)) {
                    project_speed(m, cvx, cvy, nwp, cvs, cvd);
                    okl = 1 | (clane << 1);
                    if (tab) {
                        in.tab_valid[tix] = 1; in.tab_lane[tix] = clane;
                        in.tab_s[tix] = cs; in.tab_d[tix] = cd; in.tab_vs[tix] = cvs; in.tab_vd[tix] = cvd;
                        in.tab_vx[tix] = cvx; in.tab_vy[tix] = cvy;
                    }
                } else {
                    ust |= PP_ST_CAR_UNMATCHED;
                    if (tab) in.tab_valid[tix] = 0;
                }
            } else if (sv) {                  // (tab only) a stale slot
                okl = 1 | (sln << 1);
                cs = ss; cd = sd; cvs = svs; cvd = svd;
            }
        }
        PP_TRACE_K1(3);
        if (kGroupPass && grp_or<G>((okl & 1) && id == -1 ? 1u : 0u) == 0u) {
            a.add_group<G>(P, e, T_in, (okl & 1) != 0, j, id, cs, cd, okl >> 1, cvs, cvd);
        } else {
            const int nq = iters - j0 < G ? iters - j0 : G;
            for (int q = 0; q < nq; q++) {
                const int qokl = __shfl(okl, q, G);
                const int qid = __shfl(id, q, G);
                const double qcs = __shfl(cs, q, G), qcd = __shfl(cd, q, G);
                const double qcvs = __shfl(cvs, q, G), qcvd = __shfl(cvd, q, G);
                if (qokl & 1) a.add(P, e, T_in, j0 + q, qid, qcs, qcd, qokl >> 1, qcvs, qcvd);
            }
        }
    }
    PP_TRACE_K1(4);
    status |= grp_or<G>(ust);
    // prep_finish re-reads the follow cars' velocities from the slots other lanes of the group
    // (same wave) wrote above
    if (tab) __threadfence_block();
    prep_finish<G>(in, P, pv, info, out_status, gb, S, Sv, s, v, draw, tab, r, T_in, e, a, status);
    PP_TRACE_K1(5);
}

// the grouped instantiations by name (pp_eval's launch switch)
#define PP_PREP_GRP(NAME, G)                                                                         \
    template <bool kLdsMap>                                                                         \
    __global__ __launch_bounds__(256) void NAME(MapG mg, pp_scene_batch in, pp_params P, PrepV pv,  \
                                                pp_scene_info* info, uint32_t* os, GroupBits gb) {   \
        prep_grp_body<kLdsMap, G>(mg, in, P, pv, info, os, gb);                                     \
    }
PP_PREP_GRP(k_prep_g2, 2)
PP_PREP_GRP(k_prep_g4, 4)
PP_PREP_GRP(k_prep_g8, 8)
PP_PREP_GRP(k_prep_g16, 16)
#undef PP_PREP_GRP

// ------------------------------------------------------------------------------------------------
// Phase A: control points + spline for one (scene, lane) into a slot
// ------------------------------------------------------------------------------------------------
// A slot holds one spline: knots X/Y and coefficients A/B/C (<= PP_MAX_KNOTS each) + 4 ints.
// k_cand keeps slots in LDS (stride 1); k_winner in a global scratch laid out [field][knot][S]
// (stride S: lanes of a wave touch consecutive addresses).
struct Slot {
    double *X, *Y, *A, *B, *C;
    int* meta;          // [0] n knots, [1] n control points, [2] first control-point knot, [3] flags
    int64_t st;         // element stride of the knot arrays
    int64_t mst;        // element stride of meta
    __device__ __forceinline__ double& x(int i) const { return X[i * st]; }
    __device__ __forceinline__ double& y(int i) const { return Y[i * st]; }
    __device__ __forceinline__ double& a(int i) const { return A[i * st]; }
    __device__ __forceinline__ double& b(int i) const { return B[i * st]; }
    __device__ __forceinline__ double& c(int i) const { return C[i * st]; }
    __device__ __forceinline__ int& m(int k) const { return meta[k * mst]; }
};
// k_cand's LDS slot j. PP_SLOT_AOS: knot-interleaved, knot i of slot j holds x, y, a, b, c at
// sm[(j * kKP + i) * 5 + field] — one address register per slot and immediate offsets for the five
// fields (the field-major layout needs five: in emit_paths mode they spill, and every reload waits
// for the lane's outstanding path stores). Otherwise field-major, sX[j * kKP + i] etc.
__device__ __forceinline__ Slot lds_slot(double* sX, int nslot, int* sMeta, int j) {
    (void)nslot;
    double* b = sX + (int64_t)j * kKP * 5;
    return Slot{b, b + 1, b + 2, b + 3, b + 4, sMeta + 4 * j, 5, 1};
}
constexpr int kMetaFallback = 1, kMetaTrunc = 2, kMetaWalkFail = 4;

// s: scene (inputs, stride in.n_scenes); v: its prep record (stride Sv). The spline depends on the
// ego state only (no sensor-fusion input), so every Monte-Carlo draw of a scene shares it.
__device__ void setup_lane(const MapV& m, const pp_params& P, const pp_scene_batch& in,
                           const PrepV& pv, int64_t s, int64_t v, int64_t Sv, int L, const Slot& sl) {
    const int64_t S = in.n_scenes;
    const int K = pv.K[v];
    const double pos_x = pv.pos_x[v], pos_y = pv.pos_y[v];
    const double ca = pv.ca_m[v], sa = pv.sa_m[v];
    const double start = pv.ego_speed[v], ego_d = pv.ego_d[v], ego_vd = pv.ego_vd[v];
    const int ref_wp = pv.ref_wp[v];
    const double ratio = pv.ratio[L * Sv + v];
    int flags = 0;
    // lane switch time / first control point distance (src/main.cpp:640-731)
    double min_cpd = start * 1;
    min_cpd = s_max(min_cpd, 5.0);
    const double d_diff = lane_offset(L) - ego_d;
    const double d_acc = 4;
    bool slow = false;
    double lst = 2.0;
    if ((ego_vd < 0) == (d_diff < 0)) {
        const double dmax = ego_vd * ego_vd / d_acc / 2;
        if (dmax > fabs(d_diff)) { slow = true; lst = fabs(ego_vd) / d_acc; }
    }
    if (!slow) {
        double rel = ego_vd;
        if (d_diff < 0) rel *= -1;
        const double add = fabs(d_diff);
        const double peak = sqrt(add * d_acc + rel * rel / 2);
        lst = (peak * 2 - rel) / d_acc;
    }
    double dist = start * lst;
    if (dist < 10.0) dist = 10.0;
    if (dist > 50) dist = 50;
    // knots: previous points [0, K-1) then control points, all in the local frame (:786-831)
    const int npk = K > 0 ? K - 1 : 0;
    for (int i = 0; i < npk; i++) {
        const double tx0 = in.prev_x[(int64_t)i * S + s] - pos_x;
        const double ty0 = in.prev_y[(int64_t)i * S + s] - pos_y;
        sl.x(i) = tx0 * ca - ty0 * sa;
        sl.y(i) = tx0 * sa + ty0 * ca;
    }
    // control points (:638, 744-768): first = start pose, then get_lane_pos steps
    double lx = pos_x, ly = pos_y, total = 0;
    sl.x(npk) = (pos_x - pos_x) * ca - (pos_y - pos_y) * sa;
    sl.y(npk) = (pos_x - pos_x) * sa + (pos_y - pos_y) * ca;
    int ncp = 1;
    // the five candidate control points (:744-768); their lane positions in one walk when the
    // targets are positive (always, unless the telemetry speed is not finite)
    double cpsv[5], cpx[5], cpy[5];
    bool cok[5];
    cpsv[0] = dist;
    for (int i = 1; i < 5; i++) cpsv[i] = cpsv[i - 1] + min_cpd;
    if (cpsv[0] > 0 && cpsv[1] > 0 && cpsv[2] > 0 && cpsv[3] > 0 && cpsv[4] > 0) {
        get_lane_pos_multi<5>(m, ref_wp, ratio, cpsv, L, cpx, cpy, cok);
    } else {
        for (int i = 0; i < 5; i++) get_lane_pos(m, ref_wp, ratio, cpsv[i], L, cpx[i], cpy[i], cok[i]);
    }
    for (int i = 0; i < 5; i++) {
        const double npx = cpx[i], npy = cpy[i];
        if (!cok[i]) flags |= kMetaWalkFail;
        total += sqrt((npx - lx) * (npx - lx) + (npy - ly) * (npy - ly));
        lx = npx; ly = npy;
        const double tx0 = npx - pos_x, ty0 = npy - pos_y;
        sl.x(npk + ncp) = tx0 * ca - ty0 * sa;
        sl.y(npk + ncp) = tx0 * sa + ty0 * ca;
        ncp++;
        if (total > 50 && ncp > 2) break;
    }
    int nk = npk + ncp;
    for (int i = 1; i < nk; i++) {                                      // :833-843
        if (sl.x(i) <= sl.x(i - 1)) { nk = i; flags |= kMetaTrunc; break; }
    }
    const bool fallback = nk < 3 || nk <= npk || fabs(ego_d) > 20;      // :848
    if (fallback) flags |= kMetaFallback;
    sl.m(0) = nk; sl.m(1) = ncp; sl.m(2) = npk; sl.m(3) = flags;
    if (fallback) return;
    // tk::spline::set_points (spline.h:284-373): tridiagonal band LU, rows preconditioned,
    // no pivoting. Forward sweep fuses preconditioning, Gauss step and l_solve row by row
    // (the reference's values are row-local, so the interleaving is exact);
    // temporaries: A <- scaled upper band, C <- final diagonal, B <- l_solve result.
    const int n = nk;
    double up_prev = 0, dg_prev = 1, yy_prev = 0;
    for (int i = 0; i < n; i++) {
        double lo = 0, dg, up = 0, r;
        if (i == 0) { dg = 2.0; up = 0.0; r = 0.0; }
        else if (i == n - 1) { dg = 2.0; lo = 0.0; r = 0.0; }
        else {
            const double xm = sl.x(i - 1), x0 = sl.x(i), xp = sl.x(i + 1);
            const double ym = sl.y(i - 1), y0 = sl.y(i), yp = sl.y(i + 1);
            lo = 1.0 / 3.0 * (x0 - xm);
            dg = 2.0 / 3.0 * (xp - xm);
            up = 1.0 / 3.0 * (xp - x0);
            r = (yp - y0) / (xp - x0) - (y0 - ym) / (x0 - xm);
        }
        const double sd = 1.0 / dg;                                     // saved_diag
        lo *= sd;
        up *= sd;
        dg = 1.0;
        double sum = 0;
        if (i > 0) {
            const double xx = -lo / dg_prev;                            // Gauss step k = i-1
            lo = -xx;
            dg = dg + xx * up_prev;
            sum += lo * yy_prev;                                        // l_solve
        }
        const double yy = (r * sd) - sum;
        sl.a(i) = up; sl.c(i) = dg; sl.b(i) = yy;
        up_prev = up; dg_prev = dg; yy_prev = yy;
    }
    double bb_next = 0;
    for (int i = n - 1; i >= 0; i--) {                                  // r_solve
        double sum = 0;
        if (i < n - 1) sum += sl.a(i) * bb_next;
        const double bb = (sl.b(i) - sum) / sl.c(i);
        sl.b(i) = bb;
        bb_next = bb;
    }
    for (int i = 0; i < n - 1; i++) {                                   // spline.h:345-349
        const double dx = sl.x(i + 1) - sl.x(i);
        sl.a(i) = 1.0 / 3.0 * (sl.b(i + 1) - sl.b(i)) / dx;
        sl.c(i) = (sl.y(i + 1) - sl.y(i)) / dx - 1.0 / 3.0 * (2.0 * sl.b(i) + sl.b(i + 1)) * dx;
    }
    const double h = sl.x(n - 1) - sl.x(n - 2);                         // spline.h:367-370
    sl.a(n - 1) = 0.0;
    sl.c(n - 1) = 3.0 * sl.a(n - 2) * h * h + 2.0 * sl.b(n - 2) * h + sl.c(n - 2);
}

// ------------------------------------------------------------------------------------------------
// Phase A by a team of TS threads per slot (k_cand): setup_lane's arithmetic, element for element,
// with its point- and row-local parts spread over the team and only the two band sweeps serial:
//   A1 (team)  previous-path knots; control point k: its own Map::get_lane_pos call (the reference
//              makes one call per point, :744-768) -> global xy in a(npk+1+k)/b(npk+1+k), ok in
//              c(npk+1+k), local xy in x/y(npk+1+k);
//   A2 (r = 0) the distance rule over the control points (:762), knot truncation, fallback, meta;
//   A3 (team)  each band row's preconditioned terms: a = up/dg, c = lo/dg, b = rhs/dg;
//   A4 (r = 0) Gauss + l_solve forward, r_solve backward (one division per row each way);
//   A5 (team)  the segment coefficients (spline.h:345-349) and the last row (:367-370).
// The caller puts a block barrier between the steps.
// ------------------------------------------------------------------------------------------------
struct LaneGeom {
    int K, npk, ref_wp;
    double pos_x, pos_y, ca, sa, dist, min_cpd, ratio, ego_d;
};
// (from the K1 values it reads: the build's start pose and rotation, the ego's Frenet state)
__device__ __forceinline__ LaneGeom lane_geom_from(int K, double pos_x, double pos_y, double ca_m, double sa_m,
                                                   int ref_wp, double ratio_L, double ego_d, double start,
                                                   double ego_vd, int L) {
    LaneGeom g;
    g.K = K;
    g.npk = g.K > 0 ? g.K - 1 : 0;
    g.pos_x = pos_x; g.pos_y = pos_y;
    g.ca = ca_m; g.sa = sa_m;
    g.ref_wp = ref_wp;
    g.ratio = ratio_L;
    g.ego_d = ego_d;
    double min_cpd = start * 1;
    g.min_cpd = s_max(min_cpd, 5.0);
    const double d_diff = lane_offset(L) - g.ego_d;
    const double d_acc = 4;
    bool slow = false;
    double lst = 2.0;
    if ((ego_vd < 0) == (d_diff < 0)) {
        const double dmax = ego_vd * ego_vd / d_acc / 2;
        if (dmax > fabs(d_diff)) { slow = true; lst = fabs(ego_vd) / d_acc; }
    }
    if (!slow) {
        double rel = ego_vd;
        if (d_diff < 0) rel *= -1;
        const double add = fabs(d_diff);
        const double peak = sqrt(add * d_acc + rel * rel / 2);
        lst = (peak * 2 - rel) / d_acc;
    }
    double dist = start * lst;
    if (dist < 10.0) dist = 10.0;
    if (dist > 50) dist = 50;
    g.dist = dist;
    return g;
}
__device__ __forceinline__ LaneGeom lane_geom(const PrepV& pv, int64_t v, int64_t Sv, int L) {
    return lane_geom_from(pv.K[v], pv.pos_x[v], pv.pos_y[v], pv.ca_m[v], pv.sa_m[v], pv.ref_wp[v],
                          pv.ratio[L * Sv + v], pv.ego_d[v], pv.ego_speed[v], pv.ego_vd[v], L);
}

__device__ void team_a1(const MapV& m, const pp_scene_batch& in, const LaneGeom& g, int64_t s, int L,
                        const Slot& sl, int r, int TS) {
    const int64_t S = in.n_scenes;
    for (int i = r; i < g.npk; i += TS) {
        const double tx0 = in.prev_x[(int64_t)i * S + s] - g.pos_x;
        const double ty0 = in.prev_y[(int64_t)i * S + s] - g.pos_y;
        sl.x(i) = tx0 * g.ca - ty0 * g.sa;
        sl.y(i) = tx0 * g.sa + ty0 * g.ca;
    }
    if (r == 0) {
        sl.x(g.npk) = (g.pos_x - g.pos_x) * g.ca - (g.pos_y - g.pos_y) * g.sa;
        sl.y(g.npk) = (g.pos_x - g.pos_x) * g.sa + (g.pos_y - g.pos_y) * g.ca;
    }
    for (int k = r; k < 5; k += TS) {
        double cps = g.dist;
        for (int i = 1; i <= k; i++) cps = cps + g.min_cpd;
        double px, py;
        bool ok;
        if (cps > 0) get_lane_pos_fwd<kWalkPf>(m, g.ref_wp, g.ratio, cps, L, px, py, ok);
        else get_lane_pos(m, g.ref_wp, g.ratio, cps, L, px, py, ok);
        const int j = g.npk + 1 + k;
        sl.a(j) = px; sl.b(j) = py; sl.c(j) = ok ? 1.0 : 0.0;
        const double tx0 = px - g.pos_x, ty0 = py - g.pos_y;
        sl.x(j) = tx0 * g.ca - ty0 * g.sa;
        sl.y(j) = tx0 * g.sa + ty0 * g.ca;
    }
}

__device__ void team_a2(const LaneGeom& g, const Slot& sl) {
    int flags = 0;
    double lx = g.pos_x, ly = g.pos_y, total = 0;
    int ncp = 1;
    for (int i = 0; i < 5; i++) {
        const int j = g.npk + 1 + i;
        const double npx = sl.a(j), npy = sl.b(j);
        if (sl.c(j) == 0.0) flags |= kMetaWalkFail;
        total += sqrt((npx - lx) * (npx - lx) + (npy - ly) * (npy - ly));
        lx = npx; ly = npy;
        ncp++;
        if (total > 50 && ncp > 2) break;
    }
    int nk = g.npk + ncp;
    for (int i = 1; i < nk; i++) {                                      // :833-843
        if (sl.x(i) <= sl.x(i - 1)) { nk = i; flags |= kMetaTrunc; break; }
    }
    const bool fallback = nk < 3 || nk <= g.npk || fabs(g.ego_d) > 20;  // :848
    if (fallback) flags |= kMetaFallback;
    sl.m(0) = nk; sl.m(1) = ncp; sl.m(2) = g.npk; sl.m(3) = flags;
}

// Each team lane takes a contiguous run of rows, so the slope (y(i+1) - y(i)) / (x(i+1) - x(i))
// that row i's right-hand side shares with row i+1 is divided once per run, not twice.
__device__ void team_a3(const Slot& sl, int r, int TS) {
    if (sl.m(3) & kMetaFallback) return;
    const int n = sl.m(0);
    const int per = (n + TS - 1) / TS;
    const int i0 = r * per, i1 = i0 + per < n ? i0 + per : n;
    double sl_prev = 0;                                                 // slope of segment i-1
    if (i0 > 0 && i0 < n - 1) sl_prev = (sl.y(i0) - sl.y(i0 - 1)) / (sl.x(i0) - sl.x(i0 - 1));
    for (int i = i0; i < i1; i++) {
        double lo = 0, dg, up = 0, rr;
        if (i == 0) { dg = 2.0; up = 0.0; rr = 0.0; }
        else if (i == n - 1) { dg = 2.0; lo = 0.0; rr = 0.0; }
        else {
            const double xm = sl.x(i - 1), x0 = sl.x(i), xp = sl.x(i + 1);
            const double y0 = sl.y(i), yp = sl.y(i + 1);
            lo = 1.0 / 3.0 * (x0 - xm);
            dg = 2.0 / 3.0 * (xp - xm);
            up = 1.0 / 3.0 * (xp - x0);
            const double sl_i = (yp - y0) / (xp - x0);
            rr = sl_i - sl_prev;                // (yp - y0)/(xp - x0) - (y0 - ym)/(x0 - xm)
            sl_prev = sl_i;
        }
        if (i == 0 && n > 2) sl_prev = (sl.y(1) - sl.y(0)) / (sl.x(1) - sl.x(0));
        const double sd = 1.0 / dg;                                     // saved_diag
        sl.a(i) = up * sd; sl.c(i) = lo * sd; sl.b(i) = rr * sd;
    }
}

__device__ void team_a4(const Slot& sl) {
    if (sl.m(3) & kMetaFallback) return;
    const int n = sl.m(0);
    double up_prev = 0, dg_prev = 1, yy_prev = 0;
    for (int i = 0; i < n; i++) {
        double lo = sl.c(i);
        const double up = sl.a(i);
        double dg = 1.0;
        double sum = 0;
        if (i > 0) {
            const double xx = -lo / dg_prev;                            // Gauss step k = i-1
            lo = -xx;
            dg = dg + xx * up_prev;
            sum += lo * yy_prev;                                        // l_solve
        }
        const double yy = sl.b(i) - sum;
        sl.c(i) = dg; sl.b(i) = yy;
        up_prev = up; dg_prev = dg; yy_prev = yy;
    }
    double bb_next = 0;
    for (int i = n - 1; i >= 0; i--) {                                  // r_solve
        double sum = 0;
        if (i < n - 1) sum += sl.a(i) * bb_next;
        const double bb = (sl.b(i) - sum) / sl.c(i);
        sl.b(i) = bb;
        bb_next = bb;
    }
}

__device__ void team_a5(const Slot& sl, int r, int TS) {
    if (sl.m(3) & kMetaFallback) return;
    const int n = sl.m(0);
    for (int i = r; i < n - 1; i += TS) {                               // spline.h:345-349
        const double dx = sl.x(i + 1) - sl.x(i);
        const double a = 1.0 / 3.0 * (sl.b(i + 1) - sl.b(i)) / dx;
        const double c = (sl.y(i + 1) - sl.y(i)) / dx - 1.0 / 3.0 * (2.0 * sl.b(i) + sl.b(i + 1)) * dx;
        sl.a(i) = a; sl.c(i) = c;
        if (i == n - 2) {                                               // spline.h:367-370
            const double h = sl.x(n - 1) - sl.x(n - 2);
            sl.a(n - 1) = 0.0;
            sl.c(n - 1) = 3.0 * a * h * h + 2.0 * sl.b(n - 2) * h + c;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Phase B: the resampling loop of one candidate (src/main.cpp:845-1041)
// ------------------------------------------------------------------------------------------------
// adj0/adj1: the adjusted steps 0-63 / 64-127 (two registers: an indexed pair would live in scratch)
struct CandRes { double acc_sum, travelled; int ng; uint32_t flags; uint64_t adj0, adj1; };

// Output modes. The curvature adjustment (src/main.cpp:972-1018) rotates only the local->global
// transform (centre, angle); the local path (pos_x, pos_y, arg, speed, angles) that the cost reads
// never depends on it, so a cost-only lane skips the transform, its sin/cos and the stores.
//   kOutMode 0: cost only;  2: every lane produces points;  4: the same with k_cand's cheaper
//   output-frame turn (frame_turn_at);  3: lanes with out_on RECORD their local path (pos after each step, rotation angle of each
//   curvature adjustment + a bitmask of the adjusted steps) for k_emit, which replays the
//   transform — the expensive sin/cos of the adjustments leaves the candidate loop entirely.
// Point g goes to wx[g*ws], wy[g*ws] (if wx) and px[g*ps], px[g*ps+1] (if px); in mode 3 the record
// goes to rec[g*ws] (pos_x), rec[(RN + g)*ws] (pos_y), rec[(2 RN + g)*ws] (rotation), RN = room.
// The current spline segment (bounds + coefficients) stays in registers; the segment changes every
// ~10-40 steps, so most steps read no slot memory.
template <bool kLarge, int kOutMode>
__device__ CandRes run_candidate(const pp_params& P, const Slot& sl, double cx, double cy,
                                 double angle, double ca0, double sa0, SC sc, int room, double* wx,
                                 double* wy, int64_t ws, double* px, int64_t ps, bool out_on = true,
                                 double* rec = nullptr, int dcls = 0, int64_t rs = 0) {
    (void)dcls;   // PP_DIAG builds: candidate class (|L - ego lane|) for the census
    // kOutMode 3: rec = the record base + rs (the scene), ws = the batch's scene count (rec_st)
    const bool kOut = kOutMode == 2 || kOutMode == 4;
    const bool kRec = kOutMode == 3 && out_on;
    const int64_t rstride = (int64_t)room * ws;
    CandRes R;
    R.acc_sum = 0; R.travelled = 0; R.ng = 0; R.flags = 0; R.adj0 = 0; R.adj1 = 0;
    const int nk = sl.m(0), ncp = sl.m(1), npk = sl.m(2), mflags = sl.m(3);
    if (mflags & kMetaTrunc) R.flags |= PP_ST_SPLINE_TRUNC;
    if (mflags & kMetaWalkFail) R.flags |= PP_ST_NAN;
    double pos_x = 0, pos_y = 0;
    OutFrame F = {cx, cy, ca0, sa0};
    double opx = cx, opy = cy;        // mode 4: the last output point (the frame's image of (0, 0))
    (void)angle;      // the frame turns by rotating (ca, sa) (src/main.cpp:996-997)
    double cur_t = 0.02;
    int ng = 0;
    if (mflags & kMetaFallback) {                                       // :848-901
        R.flags |= PP_ST_FALLBACK;
        const double speed = sc_get_speed(sc, cur_t);
        double cang = 0;
        int nc = 1;
        while (ng < room && nc < ncp) {
            const double dstep = speed / 50;
            const double ndx = sl.x(npk + nc) - pos_x, ndy = sl.y(npk + nc) - pos_y;
            const double cpd = sqrt(ndx * ndx + ndy * ndy);
            if (cpd < 5) { nc++; continue; }
            cur_t += 0.02;
            const double nca = ppm::atan2_fast(ndy, ndx);
            const double adiff = ppm::fmod_2pi(nca - cang + 3 * kPi) - kPi;
            const double min_radius = s_max(10.0, speed * speed / 4);
            const double rps = speed / min_radius;
            const double mas = rps / 50;
            if (fabs(adiff) > mas) {
                if (adiff > 0) cang += mas; else cang -= mas;
            } else {
                cang += adiff;
            }
            double sc_, cc_;
            ppm::sincos_pp<kLarge>(cang, sc_, cc_);
            pos_x += cc_ * dstep;
            pos_y += sc_ * dstep;
            if (kOutMode != 0 && kOut) {
                double ox, oy;
                frame_pt(F, pos_x, pos_y, ox, oy);
                if (wx && PP_CHKP(wx + ng * ws, nx, nnext, 1) && PP_CHKP(wy + ng * ws, ny, nnext, 2)) { wx[ng * ws] = ox; wy[ng * ws] = oy; }
                if (px && PP_CHKP(px + ng * ps, paths, npaths, 3) && PP_CHKP(px + ng * ps + 1, paths, npaths, 3)) st_xy(px + ng * ps, ox, oy);
            }
            if (kOutMode == 3 && kRec && PP_CHKP(rec_px(rec - rs, rstride, ng, ws, rs), rec, nrec, 4) && PP_CHKP(rec_py(rec - rs, rstride, ng, ws, rs), rec, nrec, 5)) rec_st(rec - rs, rstride, ng, ws, rs, pos_x, pos_y);
            ng++;
            R.travelled += dstep;
        }
        R.ng = ng;
        return R;
    }
    // cached segment: valid while seg_lo < x <= seg_hi (NaN x never valid)
    int cnt = -1;                    // #knots with X < x (std::lower_bound position); -1: none yet
    double seg_lo = 1.0, seg_hi = -__builtin_inf(), sx = 0, sa_ = 0, sb = 0, sc_ = 0, sy = 0;
    double arg = 0, prev_speed = sc.start;
    double uxp = 1.0, uyp = 0.0;     // previous step direction (angle 0: the local frame's x axis)
    // 1 / (target - start) for SpeedController::override_speed (constant over the walk)
#if PP_RCP1
    // (both reciprocals feed only Markstein-corrected quotients: ppm::rcp_nr1 is enough)
    const double rds = ppm::rcp_nr1(sc.target - sc.start);
    double rtt = ppm::rcp_nr1(sc.ttime);
#else
    const double rds = ppm::rcp_nr(sc.target - sc.start);
    double rtt = ppm::rcp_nr(sc.ttime);
#endif
    PP_DIAGC(20, true);     // (waves entering the loop)
#ifdef PP_LIMCENSUS
    double ref_pa = 0;      // the reference's prev_angle (src/main.cpp:906): the previous step's atan2
#endif
    // the divisions by 50 and by the ramp time: reciprocal + correction (k_cand<false>: unchecked)
#define PP_DIV50(v) (kLarge ? ppm::div_rcp(v, 50.0, 0.02) : ppm::div50_nc(v))
    // one step of the loop (src/main.cpp:911-1040): (uxp, uyp) the previous step's unit direction,
    // prev_speed its speed; the step's own go to (uxn, uyn, psn). PP_UNROLL2 runs two steps per
    // iteration with the two register sets alternating (no copies at the back edge)
    auto step = [&](const double uxp, const double uyp, const double prev_speed, double& uxn, double& uyn,
                    double& psn) __attribute__((always_inline)) {
            PP_REGION("head");
            PP_DIAGC(0, true);
            PP_DIAGC(2, !(s_max(cur_t - sc.shift, 0.0) > sc.ttime));
            double speed = sc_get_speed_r<kLarge>(sc, cur_t, rtt);
            double dstep = PP_DIV50(speed);
            const double x = arg + dstep;
            // tk::spline::operator() (spline.h:375-396)
            if (!(seg_lo < x && x <= seg_hi)) {
                PP_REGION("seg");
                // forward miss (x passed the cached segment's end; the first step starts from cnt = -1,
                // seg_hi = -inf): x(cnt) = seg_hi < x is known, so the walk resumes one knot further
                // and the bounds come from the walk's own reads — one LDS round trip for the knot and
                // one for the coefficients, instead of the two loops' re-reads
                if (__builtin_expect(x > seg_hi, 1)) {
                    double xlo = seg_hi, xhi;
                    cnt++;
                    for (;;) {
                        xhi = cnt < nk ? sl.x(cnt) : __builtin_inf();
                        if (!(xhi < x)) break;
                        xlo = xhi;
                        cnt++;
                    }
                    seg_lo = xlo;
                    seg_hi = xhi;
                    const int idx = cnt - 1 > 0 ? cnt - 1 : 0;
                    sx = cnt > 0 ? xlo : xhi;
                    sa_ = cnt == 0 ? 0.0 : sl.a(idx); sb = sl.b(idx); sc_ = sl.c(idx); sy = sl.y(idx);
                } else {
                    PP_REGION("segback");
                    PP_DIAGC(21, true);
                    if (cnt < 0) cnt = 0;
                    while (cnt < nk && sl.x(cnt) < x) cnt++;
                    while (cnt > 0 && !(sl.x(cnt - 1) < x)) cnt--;
                    const int idx = cnt - 1 > 0 ? cnt - 1 : 0;
                    seg_lo = cnt > 0 ? sl.x(cnt - 1) : -__builtin_inf();
                    seg_hi = cnt < nk ? sl.x(cnt) : __builtin_inf();
                    sx = sl.x(idx); sa_ = cnt == 0 ? 0.0 : sl.a(idx); sb = sl.b(idx); sc_ = sl.c(idx); sy = sl.y(idx);
                }
                PP_DIAGC(1, true);
            }
            PP_REGION("eval");
            const double h = x - sx;
            // the left extrapolation (cnt == 0: x <= x0) is the cubic form with a = 0 (0 h + b = b, and
            // at x == x0, h = 0 both give y0); the right one (cnt == nk) uses the last knot, whose a is
            // 0 (spline.h:367): one polynomial form for every step
            const double y = ((sa_ * h + sb) * h + sc_) * h + sy;
            double d, rd;
            const bool dok = ppm::sqrt_rd((x - pos_x) * (x - pos_x) + (y - pos_y) * (y - pos_y), d, rd);
            double acc = fabs(speed - prev_speed) * 50;
            // the turn from the previous step direction u_prev to u = (dx, dy) / d (ppm::asin_small;
            // wide turns: atan2(u_prev x u, u_prev . u)). d == 0: atan2(+0, +0) = 0, u = (1, 0).
            double ux, uy;
            {
                PP_REGION("dir");
                const double ddx = x - pos_x, ddy = y - pos_y;
                ux = ddx * rd; uy = ddy * rd;
                PP_DIAGC(18, !dok);
                if (__builtin_expect(!dok, 0)) {        // d == 0 implies !dok (q = 0 < 2^-900)
                    PP_REGION("dirfix");
                    if (d == 0) { ux = 1.0; uy = 0.0; }
                    // finite step whose squared length overflows (speeds of ~1e150 m/s and more, only
                    // in k_cand<true> scenes): rd = 0 would leave no direction, where the reference's
                    // atan2(dy, dx) still has one; normalise the step scaled by its larger component
                    if (d == __builtin_inf() && fabs(ddx) <= 0x1.fffffffffffffp1023 &&
                        fabs(ddy) <= 0x1.fffffffffffffp1023) {
                        const double m = s_max(fabs(ddx), fabs(ddy));
                        const double a = ddx / m, b = ddy / m;
                        const double n = sqrt(a * a + b * b);
                        ux = a / n; uy = b / n;
                    }
                }
            }
            PP_REGION("cross");
            const double cr = uxp * uy - uyp * ux, dt = uxp * ux + uyp * uy;
            // the reference's wrap fmod(a + 3 pi, 2 pi) - pi: for |a| <= kStepSinMax, a + 3 pi lies in
            // [2 pi, 4 pi), where fmod is the exact subtraction of 2 pi (ppm::fmod_2pi's second case)
            double adiff;
            PP_DIAGC(3, !((PP_NARROW(dt, cr)) || speed == 0));
            PP_DIAGC(8, ng == 0 && !(PP_NARROW(dt, cr)));
            PP_DIAGC(9, !(dt > 0));
            if (__builtin_expect(PP_NARROW(dt, cr), 1)) {
                PP_REGION("asin");
                adiff = (((PP_ASIN_S == 2 ? ppm::asin_small_b(cr) : PP_ASIN_S ? ppm::asin_small_s(cr) : ppm::asin_small(cr)) + 3 * kPi) - 2 * kPi) - kPi;
            } else {
                PP_REGION("wide");
                // cr, dt: components of unit vectors (finite, never both zero; NaN propagates)
                adiff = ppm::fmod_2pi_small(ppm::atan2_unit(cr, dt) + 3 * kPi) - kPi;
            }
            PP_REGION("acc");
            const double cacc = speed * 50 * fabs(adiff);
            double eff_c = cacc;
    #ifdef PP_LIMCENSUS
            bool cen_r1, cen_r2;
            {
                const double spd_r = sc_get_speed(sc, cur_t);                 // :919 (IEEE division)
                const double ast_r = ppg::atan2(y - pos_y, x - pos_x);        // :933
                const double adf_r = ppm::fmod_2pi(ast_r - ref_pa + 3 * kPi) - kPi;   // :934
                const double acc_r = fabs(spd_r - prev_speed) * 50, cacc_r = spd_r * 50 * fabs(adf_r);
                const double mx = P.maximum_acc, tol = 1e-12 * fabs(mx);
                cen_r1 = acc_r + cacc_r > mx;                                 // :941
                cen_r2 = cen_r1;
                if (cen_r1 && spd_r > prev_speed) {                           // :945-971, then :972
                    double na_r = mx - cacc_r;
                    if (na_r < 0) na_r = 0;
                    cen_r2 = na_r + cacc_r > mx;
                }
                PP_CEN(26, fabs(acc + cacc - mx) <= tol);
                PP_CEN(27, fabs(acc_r + cacc_r - mx) <= tol);
                PP_CEN(28, (acc + cacc > mx) != cen_r1);
                PP_CEN(32, __double_as_longlong(cacc) != __double_as_longlong(cacc_r));
                PP_CEN(33, __double_as_longlong(speed) != __double_as_longlong(spd_r));
                ref_pa = ast_r;
            }
    #endif
            PP_DIAGC(4, acc + cacc > P.maximum_acc);
            PP_DIAGC(10 + (ng == 0 ? 0 : ng == 1 ? 1 : ng < 5 ? 2 : ng < 10 ? 3 : ng < 20 ? 4 : 5), acc + cacc > P.maximum_acc);
            PP_DIAGC(5, acc + cacc > P.maximum_acc && speed > prev_speed);
            PP_DIAGC(7, acc + cacc > P.maximum_acc && speed > prev_speed && dcls == 1);
            if (acc + cacc > P.maximum_acc) {
                PP_REGION("lim");
                if (speed > prev_speed) {                                   // :945-971
                    PP_REGION("ovr");
                    // (inside this block acc + cacc > max held: neither is NaN; k_cand<false>'s
                    // operands are finite, so the clamp is v_max_f64)
                    double na = P.maximum_acc - cacc;
                    if (kLarge) { if (na < 0) na = 0; } else na = __builtin_fmax(na, 0.0);
                    const double ns = prev_speed + PP_DIV50(na);
                    sc_override_r<kLarge>(sc, cur_t, ns, rds);
                    speed = ns;
                    sc.ttime += 0.02;
                    rtt = PP_RCP1 ? ppm::rcp_nr1(sc.ttime) : ppm::rcp_nr(sc.ttime);
                    dstep = PP_DIV50(speed);
                    acc = na;
                    R.flags |= PP_ST_ACC_OVERRIDE;
                }
                PP_DIAGC(6, acc + cacc > P.maximum_acc);
                PP_CEN(29, true);
                PP_CEN(30, fabs(acc + cacc - P.maximum_acc) <= 1e-12 * fabs(P.maximum_acc));
                PP_CEN(31, cen_r1 && (acc + cacc > P.maximum_acc) != cen_r2);
                PP_REGION("lim2");
                if (acc + cacc > P.maximum_acc) {                           // :972-1018
                    PP_REGION("adj");
                    double nc = P.maximum_acc - acc;
                    if (kLarge) { if (nc < 0) nc = 0; } else nc = __builtin_fmax(nc, 0.0);
                    if (kOutMode == 2) {
                        // the output frame turns about the current point (src/main.cpp:986-997)
                        double cr, sr;
                        turn_sincos<kLarge>(turn_angle<kLarge>(nc, speed, adiff), sr, cr);
                        frame_turn(F, pos_x, pos_y, cr, sr);
                    } else if (kOutMode == 4) {
    #if PP_PATHS_INC
                        PP_DIAGC(19, !(!kLarge && PP_NARROW(dt, cr)));
                        PP_DIAGC(23, !kLarge && PP_NARROW(dt, cr));
                        if (!kLarge && PP_NARROW(dt, cr)) {
                            PP_REGION("adjn");
                            turn_narrow(F.ca, F.sa, nc, speed, adiff, dt, cr);
                        } else {
                            PP_REGION("adjwide");
                            double crr, srr;
                            turn_sincos<kLarge>(kLarge ? turn_angle<true>(nc, speed, adiff)
                                                       : turn_angle_fast(nc, speed, adiff), srr, crr);
                            frame_rot(F.ca, F.sa, crr, srr);
                        }
    #else
                        double cr, sr;
                        turn_sincos<kLarge>(turn_angle_fast(nc, speed, adiff), sr, cr);
                        frame_turn_at(F, pos_x, pos_y, opx, opy, cr, sr);
    #endif
                    }
                    if (kOutMode == 3 && kRec) {
                        // the turn angle for k_emit's replay of the output frame
                        double* rp = rec_rot(rec - rs, rstride, ng, ws, rs);
                        if (PP_CHKP(rp, rec, nrec, 6))
                            PP_ST(rp, turn_angle<kLarge>(nc, speed, adiff));   // rot (src/main.cpp:986)
                        const uint64_t bit = 1ull << (ng & 63);
                        if (ng < 64) R.adj0 |= bit; else R.adj1 |= bit;
                    }
                    eff_c = nc;
                    R.flags |= PP_ST_CURV_ADJUST;
                }
            }
            PP_REGION("tail");
            cur_t += 0.02;
            psn = speed;
            uxn = ux; uyn = uy;
            double sp_step, dpy;
            if (kLarge) {
                sp_step = ppm::div_rcp_n((x - pos_x) * dstep, d, rd, dok);
                dpy = ppm::div_rcp_n((y - pos_y) * dstep, d, rd, dok);
            } else {          // ppm::div_rcp_d for both numerators, one !dok branch
                const double nx = (x - pos_x) * dstep, ny = (y - pos_y) * dstep;
                const double qx = nx * rd, qy = ny * rd;
                sp_step = __builtin_fma(__builtin_fma(-qx, d, nx), rd, qx);
                dpy = __builtin_fma(__builtin_fma(-qy, d, ny), rd, qy);
                if (__builtin_expect(!dok, 0)) { PP_REGION("tailfix"); sp_step = nx / d; dpy = ny / d; }
            }
            PP_REGION("tail2");
            pos_y += dpy;
            arg += sp_step;
            pos_x = arg;      // == pos_x + sp_step: both start at 0 and add the same sp_step (:1027-1031)
            if (kOutMode != 0 && kOut) {
                PP_REGION("out");
                PP_DIAGC(22, wx != nullptr);
                double ox, oy;
    #if PP_PATHS_INC
                if (kOutMode == 4) { ox = opx; oy = opy; frame_step(F.ca, F.sa, sp_step, dpy, ox, oy); }
    #else
                if (kOutMode == 4) frame_pt_fma(F, pos_x, pos_y, ox, oy);
    #endif
                else frame_pt(F, pos_x, pos_y, ox, oy);
                if (wx && PP_CHKP(wx + ng * ws, nx, nnext, 1) && PP_CHKP(wy + ng * ws, ny, nnext, 2)) { PP_REGION("outw"); wx[ng * ws] = ox; wy[ng * ws] = oy; }
                PP_REGION("out2");
                if (px && PP_CHKP(px + ng * ps, paths, npaths, 3) && PP_CHKP(px + ng * ps + 1, paths, npaths, 3))
                    st_xy(px + ng * ps, ox, oy);      // one 16-B store (x, y)
                if (kOutMode == 4) { opx = ox; opy = oy; }
            }
            if (kOutMode == 3 && kRec && PP_CHKP(rec_px(rec - rs, rstride, ng, ws, rs), rec, nrec, 4) && PP_CHKP(rec_py(rec - rs, rstride, ng, ws, rs), rec, nrec, 5)) rec_st(rec - rs, rstride, ng, ws, rs, pos_x, pos_y);
            PP_REGION("latch");
            ng++;
            R.acc_sum += acc + eff_c;
            R.travelled += dstep;
        };
#if PP_UNROLL2
    double uxq = 0, uyq = 0, psq = 0;
    while (arg < 50 && ng < room) {
        step(uxp, uyp, prev_speed, uxq, uyq, psq);
        if (!(arg < 50 && ng < room)) break;
        step(uxq, uyq, psq, uxp, uyp, prev_speed);
#if PP_UNROLL2 > 1
        if (!(arg < 50 && ng < room)) break;
        step(uxp, uyp, prev_speed, uxq, uyq, psq);
        if (!(arg < 50 && ng < room)) break;
        step(uxq, uyq, psq, uxp, uyp, prev_speed);
#endif
    }
#else
    while (arg < 50 && ng < room) step(uxp, uyp, prev_speed, uxp, uyp, prev_speed);
#endif
    PP_REGION("end");
    R.ng = ng;
    return R;
}

// per-candidate cost (identical formula in oracle/pp_oracle.c cand_cost)
__device__ __forceinline__ double cand_cost(const pp_params& P, const CandRes& R, int K, double score_L,
                                            int L, int T, double v, int open_mask, int ego_lane,
                                            uint32_t& flags) {
    const double acc_mean = R.ng > 0 ? R.acc_sum / R.ng : 0.0;
    const double ideal = (P.n_points - K) * P.max_speed / 50;
    const double deficit = 1.0 - R.travelled / ideal;
    double J = (2.5 - score_L) + acc_mean / P.maximum_acc + deficit + ((R.flags & PP_ST_FALLBACK) ? 1.0 : 0.0);
    if (!(J == J) || (R.flags & PP_ST_NAN)) { J = 999.0; flags |= PP_ST_NAN; }
    if (J > 999.0) J = 999.0;
    if (J < 0.0) J = 0.0;
    if (P.cost_mode == PP_COST_REFERENCE) {
        if (L != T) J += 1e6;
        if (v != P.max_speed) J += 1e3;
    } else {
        if (!((open_mask >> L) & 1) && L != ego_lane) J += 10.0;
    }
    return J;
}

__device__ __forceinline__ SC make_sc(const pp_params& P, const PrepV& pv, int64_t S, int64_t s,
                                      int L, double v) {
    SC sc;                                        // SpeedController ctor (src/main.cpp:495-502)
    sc.shift = 0;
    sc.start = pv.ego_speed[s];
    sc.target = v;
    sc.ttime = fabs(sc.start - v) / P.relaxed_acc;
    const int lm = pv.lim_mask[s];
    if (lm & 1) sc_add_limit(sc, pv.in_ts[s], pv.in_tt[s]);            // :1425-1431
    if (lm & (2 << L)) sc_add_limit(sc, pv.l_ts[L * S + s], pv.l_tt[L * S + s]);  // :1432-1438
    return sc;
}


// K4 inside k_cand (reference mode, emit_in): the winner lane of scene s replays the output
// transform of its recorded path (src/main.cpp:994-1007, 1033-1037) with the sin/cos of each
// recorded turn already in LDS (pcr/psr, one entry per step, computed by the block's team as
// emit_scene computes them): only the chain of turns and points is left to the lane. Operations
// and order are emit_scene's, so the outputs are bit-identical to the k_emit path.
template <int kChunk>
__device__ __forceinline__ void emit_scene_pre(const pp_scene_batch& in, const pp_params& P,
                                               const PrepV& pv, const pp_result& out, const double* rec,
                                               int64_t s, int K, int ng, uint64_t m0, uint64_t m1,
                                               const double* pcr, const double* psr) {
    const int64_t S = in.n_scenes;
    const int N = P.n_points;
    const int64_t rstride = (int64_t)(N - K) * S;
    {   // the kept previous points: every load issued before the first store
        double kx[PP_PREV_KEEP], ky[PP_PREV_KEEP];
#pragma unroll
        for (int i = 0; i < PP_PREV_KEEP; i++)
            if (i < K) { kx[i] = in.prev_x[(int64_t)i * S + s]; ky[i] = in.prev_y[(int64_t)i * S + s]; }
#pragma unroll
        for (int i = 0; i < PP_PREV_KEEP; i++)
            if (i < K) { PP_ST(out.next_x + (int64_t)i * S + s, kx[i]); PP_ST(out.next_y + (int64_t)i * S + s, ky[i]); }
    }
    OutFrame F = {pv.pos_x[s], pv.pos_y[s], pv.ca_p[s], pv.sa_p[s]};
    double pxp = 0, pyp = 0;                       // local position before the step
    for (int g0 = 0; g0 < ng; g0 += kChunk) {
        double px_[kChunk], py_[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int g = g0 + u;
#ifdef PP_CHECK
            if (g < ng) { PP_CHKP(rec_py((double*)rec, rstride, g, S, s), rec, nrec, 19); }
#endif
            px_[u] = 0.0; py_[u] = 0.0;
            if (g < ng) rec_ld(rec, rstride, g, S, s, px_[u], py_[u]);
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int g = g0 + u;
            if (g >= ng) break;
            if ((g < 64 ? (m0 >> g) & 1 : (m1 >> (g - 64)) & 1) != 0) frame_turn(F, pxp, pyp, pcr[g], psr[g]);
            double ox, oy;
            frame_pt(F, px_[u], py_[u], ox, oy);
            if (!PP_CHKP(out.next_x + (int64_t)(K + g) * S + s, nx, nnext, 17)) break;
            PP_ST(out.next_x + (int64_t)(K + g) * S + s, ox);
            PP_ST(out.next_y + (int64_t)(K + g) * S + s, oy);
            pxp = px_[u];
            pyp = py_[u];
        }
    }
    for (int i = K + ng; i < N; i++) { out.next_x[(int64_t)i * S + s] = 0; out.next_y[(int64_t)i * S + s] = 0; }
}

// ------------------------------------------------------------------------------------------------
// K2: candidates. One workgroup = SPB scenes x C candidates; slots in LDS.
// kSlow = false: every scene except those flagged kLimSlow by k_prep (no library call in the
// loop, so the register peak stays at the loop's own state); kSlow = true: only flagged scenes.
// kMode 2: every candidate writes its path (emit_paths); 1: reference mode, the winner lanes
// write next_x/next_y; 0: cost only (comfort mode; k_winner produces the outputs).
// ------------------------------------------------------------------------------------------------
// One group g of the candidate grid (BPS == 1: scenes [g SPB, g SPB + SPB); BPS > 1: candidates
// [coff, coff + 256) of scene g / BPS) by the whole workgroup. Every barrier inside is reached by
// all threads of the block (the early return is block-uniform).
// kEmitIn (reference mode, kMode 1): 0 the winners' paths are replayed by k_emit; 1 by the block
// after phase B (K4 in the block, below); 2 the winner lanes write their points during the loop
// (output mode 2: the transform and its turns in the step, no record and no replay — the
// single-frame and small-batch step, whose time is the winners' serial chain)
// kPreA: the block's (single) scene has its fast-path spline slots built already (k_plan_frame's
// second wave builds them while the first runs K1): phase A is skipped
#ifndef PP_WSLOT
#define PP_WSLOT 1            // 0: k_winner makes the decision and builds the winner's spline (A/B)
#endif
// k_winner's blocks and spline slots (kWinKnots = 9 previous + 6 control points, the real maximum)
constexpr int kWinBlock = 64;
constexpr int kWinKnots = 15;
static_assert(PP_PREV_KEEP - 1 + 6 <= kWinKnots && kWinKnots <= kKP, "slot too small");
constexpr int kWinRec = 5 * kWinKnots + 3;    // stored winner slot per scene (doubles): knots, 4 meta ints, pad (16-B records)
template <bool kSlow, int kMode, int kEmitIn = 0, bool kPreA = false>
__device__ __forceinline__ void cand_group(const MapG& mg, const pp_scene_batch& in, const pp_params& P,
                                           const PrepV& pv, const pp_result& out, int SPB, int BPS,
                                           double* rec, uint64_t* adjm, int64_t g, double* sm,
                                           double* wslot = nullptr) {
    constexpr bool emit_in = kEmitIn == 1 && kMode == 1;
    constexpr bool win_inline = kEmitIn == 2 && kMode == 1;
    const int NS = P.n_speeds, Cv = NL * NS, N = P.n_points;
    const int D = P.n_draws > 1 ? P.n_draws : 1;
    const int C = D * Cv;                     // candidates per scene (all draws)
    const int nslot = NL * SPB;
    double* sX = sm;
    double* sY = sX + nslot * kKP;
    double* sA = sY + nslot * kKP;
    double* sB = sA + nslot * kKP;
    double* sC = sB + nslot * kKP;
    int* sMeta = (int*)(sC + nslot * kKP);
    uint32_t* sFlags = (uint32_t*)(sMeta + 4 * nslot);
    const MapV m = map_view(mg.buf, mg.n);
    const int64_t S = in.n_scenes;
    const int64_t Sv = S * D;
    // block -> scenes: BPS == 1: SPB whole scenes; BPS > 1 (C > 256): one scene, candidates
    // [coff, coff + 256) of it; BPS < 0 (kMode 2, the flat geometry): the batch's candidates
    // [256 g, 256 g + 256), from candidate coff of scene s0 on, over at most SPB scenes
    int64_t s0;
    int coff;
    int nsc;
    if (BPS == 1) { s0 = g * SPB; coff = 0; }
    else if (BPS < 0) { s0 = g * 256 / C; coff = (int)(g * 256 - s0 * C); }
    else { s0 = g / BPS; coff = (int)(g - s0 * BPS) * 256; }
    if (BPS < 0) {
        const int span = (coff + 255) / C + 1;
        nsc = (int)((S - s0) < span ? (S - s0) : span);
    } else {
        nsc = (int)((S - s0) < SPB ? (S - s0) : SPB);
    }
    const int tid = threadIdx.x;
    // per scene: any of its draws flagged kLimSlow (absurd heading, or a speed or ramp time outside
    // the range of the unchecked divisions) -> the scene runs in the k_cand<true> instantiation
    uint32_t* sSlow = sFlags + SPB;
    // kMode 1 with emit_in: each winner's step count and adjusted-step masks for the in-block K4
    uint64_t* sAdj = (uint64_t*)(((uintptr_t)(sSlow + SPB) + 7) & ~(uintptr_t)7);
    int* sNg = (int*)(sAdj + 2 * SPB);
    // comfort mode with a stored winner slot: each lane's cost (the host sizes the LDS for it)
    double* sCost = (double*)(((uintptr_t)(sNg + SPB) + 7) & ~(uintptr_t)7);
    if (tid < SPB) { sFlags[tid] = 0; sSlow[tid] = 0; }
#ifdef PP_TRACE
    if (!kSlow && tid == 0) {
        PP_TRACE_AT(blockIdx.x, 0);
        if (blockIdx.x < (unsigned)kTraceK1) g_trace[8 * blockIdx.x + 7] = trace_hwid();
    }
#endif
#ifdef PP_CHECK
    if (!kPreA) {
        for (int i = tid; i < 5 * nslot * kKP; i += (int)blockDim.x) sX[i] = __builtin_nan("");
        for (int i = tid; i < 4 * nslot; i += (int)blockDim.x) sMeta[i] = kMetaPoison;
    }
#endif
    __syncthreads();
    bool mine = false;
    for (int t = tid; t < nsc * D; t += (int)blockDim.x) {
        const int q = t / D;
        if (pv.lim_mask[(s0 + q) * D + (t - q * D)] & kLimSlow) { atomicOr(&sSlow[q], 1u); mine = true; }
    }
    if (!__syncthreads_or(mine) && kSlow) return;      // whole block leaves: no flagged scene
    if (!kPreA) {   // phase A: a team of TS threads per slot (team_a1..a5), block barriers between the steps
        int TS = (int)blockDim.x / nslot;
        if (TS > 8) TS = 8;
        const int j = tid / TS, r = tid - j * TS;
        const bool act = j < NL * nsc && ((sSlow[j / NL] != 0) == kSlow);
        const Slot sl = lds_slot(sX, nslot, sMeta, j);
        const int L = j % NL;
        const int64_t s = s0 + j / NL;
        LaneGeom g;
        PP_REGION_A("a1");
#ifndef PP_SKIP_A1
        if (act) { g = lane_geom(pv, s * D, Sv, L); team_a1(m, in, g, s, L, sl, r, TS); }
#endif
        __syncthreads();
        PP_REGION_A("a2");
        // the two serial steps (A2, A4) on one lane per slot, slots in lane order: NL * SPB <= 64
        // slots fit the block's first wave, whose instruction stream is then the only one paying
        // for them (a team layout spreads them over every wave of the block)
        const int js = tid;
        const bool act_s = js < NL * nsc && ((sSlow[js / NL] != 0) == kSlow);
        const Slot sls = lds_slot(sX, nslot, sMeta, js);
        if (act_s) {
            const int64_t vs = (s0 + js / NL) * D;
            LaneGeom gs;
            gs.K = pv.K[vs];
            gs.npk = gs.K > 0 ? gs.K - 1 : 0;
            gs.pos_x = pv.pos_x[vs]; gs.pos_y = pv.pos_y[vs]; gs.ego_d = pv.ego_d[vs];
#ifndef PP_SKIP_A2
            team_a2(gs, sls);
#endif
        }
        __syncthreads();
        PP_REGION_A("a3");
#ifndef PP_SKIP_A3
        if (act) team_a3(sl, r, TS);
#endif
        __syncthreads();
        PP_REGION_A("a4");
#ifndef PP_SKIP_A4
        if (act_s) team_a4(sls);
#endif
        __syncthreads();
        PP_REGION_A("a5");
#ifndef PP_SKIP_A5
        if (act) team_a5(sl, r, TS);
#endif
    }
    PP_REGION_A("pre");
    __syncthreads();
    if (!kSlow && tid == 0) PP_TRACE_AT(blockIdx.x, 1);
    // Lane -> candidate. Reference mode without draws (kMode 1): lanes [0, nsc) run the scenes'
    // winning candidates (planner lane T, max_speed: known from k_prep) and record their paths;
    // lanes >= nsc run the C - 1 other candidates of each scene cost-only. The output work is
    // thereby confined to the block's first wave; the other waves run the lean cost-only loop.
    int sc_l, c;
    if (kMode == 1) {
        if (tid < nsc) {
            sc_l = tid;
            c = pv.T[s0 + tid] * NS;
        } else {
            const int t2 = tid - nsc;
            sc_l = t2 / (C - 1);
            const int r = t2 - sc_l * (C - 1);
            const int cw = sc_l < nsc ? pv.T[s0 + sc_l] * NS : 0;
            c = r < cw ? r : r + 1;
        }
    } else {
        const int t = tid + coff;
        sc_l = t / C;
        c = t - sc_l * C;
    }
    if (sc_l < nsc && c < C && ((sSlow[sc_l] != 0) == kSlow)) {   // phase B
        const int64_t s = s0 + sc_l;
        const int d = c / Cv, cc = c - d * Cv;
        const int64_t v = s * D + d;              // this draw's prep record
        const int L = cc / NS, k = cc - L * NS;
        const int j = sc_l * NL + L;
        const Slot sl = lds_slot(sX, nslot, sMeta, j);
#ifdef PP_CHECK
        {   // the slot was written by this group's phase A (not left over from an earlier group)
            const int nk_ = sl.m(0), ncp_ = sl.m(1), npk_ = sl.m(2);
            chk_(j < nslot && nk_ != kMetaPoison && nk_ >= 1 && nk_ <= kKP && ncp_ >= 1 && ncp_ <= 6 &&
                 npk_ >= 0 && npk_ < PP_PREV_KEEP, 20, j, g);
        }
#endif
        const double vt = cand_speed(P, pv.ego_speed[v], k);
        const SC sc = make_sc(P, pv, Sv, v, L, vt);
        const int K = pv.K[v], T = pv.T[v];
        // reference mode: the winning candidate (planner lane, max_speed) is known before the
        // loop, so its lane writes next_x/next_y (point-major) during the same pass
        const bool winner = kMode == 1 ? tid < nsc
                                       : (kMode == 2 && P.cost_mode == PP_COST_REFERENCE && L == T && k == 0);
        CandRes R;
        if (kMode == 2) {
            // every candidate writes its path; in reference mode the winner also writes next_x/y
            double* wx = nullptr;
            double* wy = nullptr;
            if (winner) {
                for (int i = 0; i < K; i++) {
                    if (!PP_CHKP(out.next_x + (int64_t)i * S + s, nx, nnext, 9)) break;
                    out.next_x[(int64_t)i * S + s] = in.prev_x[(int64_t)i * S + s];
                    out.next_y[(int64_t)i * S + s] = in.prev_y[(int64_t)i * S + s];
                }
                wx = out.next_x + (int64_t)K * S + s;
                wy = out.next_y + (int64_t)K * S + s;
            }
            const int64_t ps = (int64_t)C * 2;
            double* p0 = out.paths + ((s * N) * C + c) * 2;
            for (int i = 0; i < K; i++) {
                if (!PP_CHKP(p0 + i * ps + 1, paths, npaths, 7)) break;
                st_xy(p0 + i * ps, in.prev_x[(int64_t)i * S + s], in.prev_y[(int64_t)i * S + s]);
            }
            double* px = p0 + K * ps;
#ifdef PP_DIAG_NOB
            // diagnostic builds only: phase B skipped (wrong results; measures everything else)
            R = CandRes{0, 0, N - K, 0, 0, 0};
            (void)sc; (void)wx; (void)wy;
#else
            R = run_candidate<kSlow, 4>(P, sl, pv.pos_x[v], pv.pos_y[v], pv.angle[v],
                                                       pv.ca_p[v], pv.sa_p[v], sc, N - K, wx, wy, S,
                                                       px, ps);
#endif
            for (int i = R.ng; i < N - K; i++) {
                if (!PP_CHKP(px + i * ps + 1, paths, npaths, 8)) break;
                st_xy(px + i * ps, __builtin_nan(""), __builtin_nan(""));
            }
            if (out.path_len && PP_CHK(s * C + c < g_lim.ncost, 11, s * C + c)) out.path_len[s * C + c] = K + R.ng;
            if (winner) {
                for (int i = K + R.ng; i < N; i++) {
                    if (!PP_CHKP(out.next_x + (int64_t)i * S + s, nx, nnext, 10)) break;
                    out.next_x[(int64_t)i * S + s] = 0; out.next_y[(int64_t)i * S + s] = 0;
                }
                out.n_out[s] = K + R.ng;
                out.winner[s] = c;
            }
        } else if (win_inline && tid < 64) {
            // reference mode, the block's first wave: the winners write next_x/next_y in the loop
            // (the rest of the wave runs the same instantiation without outputs, in lockstep)
            double* wx = nullptr;
            double* wy = nullptr;
            if (winner) {
                for (int i = 0; i < K; i++) {
                    if (!PP_CHKP(out.next_x + (int64_t)i * S + s, nx, nnext, 9)) break;
                    out.next_x[(int64_t)i * S + s] = in.prev_x[(int64_t)i * S + s];
                    out.next_y[(int64_t)i * S + s] = in.prev_y[(int64_t)i * S + s];
                }
                wx = out.next_x + (int64_t)K * S + s;
                wy = out.next_y + (int64_t)K * S + s;
            }
            R = run_candidate<kSlow, 2>(P, sl, pv.pos_x[v], pv.pos_y[v], pv.angle[v], pv.ca_p[v], pv.sa_p[v],
                                        sc, N - K, wx, wy, S, nullptr, 0);
            if (winner) {
                for (int i = K + R.ng; i < N; i++) {
                    if (!PP_CHKP(out.next_x + (int64_t)i * S + s, nx, nnext, 10)) break;
                    out.next_x[(int64_t)i * S + s] = 0; out.next_y[(int64_t)i * S + s] = 0;
                }
                out.n_out[s] = K + R.ng;
                out.winner[s] = c;
            }
        } else if (kMode == 1 && tid < 64) {
            // reference mode, the block's first wave: the winners record their local path
            // (3 stores per step) for k_emit; the other lanes of the wave are cost-only
#ifdef PP_DIAG_NOB
            R = CandRes{0, 0, N - K, 0, 0, 0};   // (diagnostic builds: phase B skipped)
#else
            R = run_candidate<kSlow, 3>(P, sl, 0, 0, 0, 1, 0, sc, N - K, nullptr, nullptr,
                                                       S, nullptr, 0, winner, rec + s, 0, s);
#endif
            if (winner && emit_in) {          // in-block K4 below: step count and masks in LDS
                out.n_out[s] = K + R.ng;
                out.winner[s] = c;
                sNg[sc_l] = R.ng; sAdj[2 * sc_l] = R.adj0; sAdj[2 * sc_l + 1] = R.adj1;
            } else if (winner && PP_CHK(s < g_lim.nscen, 12, s) && PP_CHKP(adjm + S + s, adjm, nadj, 13)) {
                out.n_out[s] = K + R.ng;
                out.winner[s] = c;
                adjm[s] = R.adj0;
                adjm[S + s] = R.adj1;
            }
        } else {
#ifdef PP_DIAG_NOB
            R = CandRes{0, 0, N - K, 0, 0, 0};   // (diagnostic builds: phase B skipped)
#else
            R = run_candidate<kSlow, 0>(P, sl, 0, 0, 0, 1, 0, sc, N - K,
                                                       nullptr, nullptr, 0, nullptr, 0, true, nullptr,
                                                       fabs(sc.target - sc.start) >= 7.5 * sc.ttime ? 2 : (sc.target > sc.start ? 1 : 0));
#endif
        }
        PP_REGION_A("post");
        uint32_t flags = R.flags;
        const double cost = cand_cost(P, R, K, pv.score[L * Sv + v], L, T, vt, pv.open_mask[v],
                                      pv.ego_lane[v], flags);
        if (PP_CHKP(out.cost + s * C + c, cost, ncost, 14)) out.cost[s * C + c] = cost;
        if (kMode == 0 && wslot && BPS == 1 && D == 1) sCost[tid] = cost;     // (k_winner_st's decision)
        if (D > 1) flags |= (uint32_t)pv.status[v];     // every draw's planner flags
        atomicOr(&sFlags[sc_l], flags);
    }
    if (!kSlow && (tid & 63) == 0 && tid < 256) PP_TRACE_AT(blockIdx.x, 2 + (tid >> 6));
    __syncthreads();
    if (tid < nsc && ((sSlow[tid] != 0) == kSlow) && PP_CHK(s0 + tid < g_lim.nscen, 15, s0 + tid)) {
        const uint32_t st = (uint32_t)pv.status[(s0 + tid) * D] | sFlags[tid];
        if (BPS == 1) out.status[s0 + tid] = st;
        else atomicOr(&out.status[s0 + tid], st);     // zeroed by k_prep
    }
    if (!kSlow && tid == 0) PP_TRACE_AT(blockIdx.x, 6);
    if (kMode == 0 && wslot && BPS == 1 && D == 1) {
        // comfort mode (every candidate of the block's scenes in this block, no draws): the
        // per-scene decision, k_winner's rule (first minimum over (lane, speed)) over the costs the
        // lanes left in LDS, then the winner's spline slot copied from LDS to the stored-slot buffer,
        // so k_winner_st re-runs the winner without building its spline a second time (the slot is
        // what setup_lane builds, element for element)
        int* sBest = sNg;
        if (tid < nsc && ((sSlow[tid] != 0) == kSlow)) {
            int best = 0;
            double bc = 0;
            for (int cc = 0; cc < Cv; cc++) {
                const double cst = sCost[tid * C + cc];
                if (cc == 0 || cst < bc) { bc = cst; best = cc; }
            }
            sBest[tid] = best;
            out.winner[s0 + tid] = best;
        }
        __syncthreads();
        // the scene's record: the LDS slot's knot-interleaved doubles (x, y, a, b, c of knot i at
        // 5 i + field) as they lie, then the 4 meta ints; consecutive threads copy consecutive
        // items of a scene, so a wave stores contiguous bytes
        constexpr int kItems = 5 * kWinKnots + 4;
        for (int idx = tid; idx < nsc * kItems; idx += (int)blockDim.x) {
            const int w = idx / kItems, e = idx - w * kItems;
            if ((sSlow[w] != 0) != kSlow) continue;
            const int64_t s = s0 + w;
            const Slot sl = lds_slot(sX, nslot, sMeta, w * NL + sBest[w] / NS);
            double* rec_s = wslot + s * kWinRec;
            if (e < 5 * kWinKnots) rec_s[e] = sl.X[e];
            else ((int*)(rec_s + 5 * kWinKnots))[e - 5 * kWinKnots] = sl.m(e - 5 * kWinKnots);
        }
    }
    if (kMode == 1 && emit_in) {
        // K4 in the block (reference mode): the spline slots are free now, so the team computes
        // the sin/cos of every recorded turn of the block's winners into them (one item per
        // winner x step), then each winner lane replays its transform from its own record
        // (emit_scene_pre: the chain of turns and points only, emit_scene's operations).
        double* pcr = sm;
        double* psr = sm + SPB * N;               // 2 SPB N <= 5 NL SPB kKP doubles (host: emit_in)
        for (int idx = tid; idx < nsc * N; idx += (int)blockDim.x) {
            const int w = idx / N, gs = idx - w * N;
            if (((sSlow[w] != 0) != kSlow) || gs >= sNg[w]) continue;
            const uint64_t mm = gs < 64 ? sAdj[2 * w] : sAdj[2 * w + 1];
            if (!((mm >> (gs & 63)) & 1)) continue;
            const int64_t s = s0 + w;
            const double* rr = rec_rot(rec, (int64_t)(N - pv.K[s]) * S, gs, S, s);
            if (!PP_CHKP(rr, rec, nrec, 18)) continue;
            const double rt = *rr;
            double sr, cr;
            turn_sincos<true>(rt, sr, cr);
            pcr[idx] = cr; psr[idx] = sr;
        }
        __syncthreads();
        if (!kSlow && tid == 0) PP_TRACE_AT(blockIdx.x, 7);
        if (tid < nsc && ((sSlow[tid] != 0) == kSlow)) {
            const int64_t s = s0 + tid;
            emit_scene_pre<kEmitChunk>(in, P, pv, out, rec, s, pv.K[s], sNg[tid], sAdj[2 * tid],
                                          sAdj[2 * tid + 1], pcr + tid * N, psr + tid * N);
        }
    }
}

// k_cand<false>: the full grid, one group per workgroup; scenes k_prep flagged kLimSlow are left
// to k_cand<true>, which runs only the groups whose bit k_prep set in `gbits` (a bitmap over the
// groups): gridDim.x workgroups walk the bitmap with stride gridDim.x (the bit test and the loop
// are block-uniform; a barrier separates consecutive groups' use of the block's LDS). Each group
// clears its bit after use, so the bitmap is all zero again for the next pp_eval.
template <bool kSlow, int kMode>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kMode == 2 ? PP_CAND_WAVES2 : kCandWaves))) void k_cand(MapG mg, pp_scene_batch in, pp_params P, PrepV pv,
                                              pp_result out, int SPB, int BPS, double* rec, uint64_t* adjm,
                                              uint32_t* gbits, int64_t ngroups, const uint32_t* glist,
                                              const uint32_t* gcount, int64_t g0, double* wslot) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (!kSlow) {
        cand_group<false, kMode>(mg, in, P, pv, out, SPB, BPS, rec, adjm, g0 + blockIdx.x, sm, wslot);
        return;
    }
    // the flagged groups k_prep listed (each listed once: the first setter of its bit appends it)
    const uint32_t nl = *gcount;                                  // same address for every lane
    for (uint32_t i = blockIdx.x; i < nl; i += gridDim.x) {
        const int64_t g = glist[i];
        if (!PP_CHK(g < ngroups, 21, g)) continue;               // (never: k_prep lists this call's groups)
        __syncthreads();                                          // the previous group's LDS readers are done
        cand_group<true, kMode>(mg, in, P, pv, out, SPB, BPS, rec, adjm, g, sm, wslot);
        if (threadIdx.x == 0) atomicAnd(&gbits[g >> 5], ~(1u << (g & 31)));
    }
}

// ------------------------------------------------------------------------------------------------
// K3: per-scene winner: argmin over the candidate costs (first minimum, as the oracle; with
// Monte-Carlo draws over the draw-averaged cost of each (lane, speed)), then the winning
// candidate re-run on the nominal scene with outputs.
// One lane per scene, 64 scenes per block; each lane's spline slot lives in LDS (kWinKnots =
// 9 previous + 6 control points, the real maximum) so 4 blocks fit a CU; with the segment cache
// the loop rarely reads it. next_x/next_y are point-major ([i * S + s], the batch's own
// convention): every step of the wave stores 512 contiguous bytes.
// ------------------------------------------------------------------------------------------------
// the winner's re-run with outputs (best: its candidate index; sl: its spline slot, built)
template <bool kSlow>
__device__ __forceinline__ void winner_run(const pp_scene_batch& in, const pp_params& P, const PrepV& pv,
                                           const pp_result& out, int64_t s, int64_t v0, int64_t Sv,
                                           int best, const Slot& sl) {
    const int64_t S = in.n_scenes;
    const int NS = P.n_speeds, N = P.n_points;
    const int L = best / NS, k = best - L * NS;
    const double v = cand_speed(P, pv.ego_speed[v0], k);
    const SC sc = make_sc(P, pv, Sv, v0, L, v);
    const int K = pv.K[v0];
    for (int i = 0; i < K; i++) {
        out.next_x[(int64_t)i * S + s] = in.prev_x[(int64_t)i * S + s];
        out.next_y[(int64_t)i * S + s] = in.prev_y[(int64_t)i * S + s];
    }
    const CandRes R = run_candidate<kSlow, 2>(P, sl, pv.pos_x[v0], pv.pos_y[v0], pv.angle[v0],
                                                    pv.ca_p[v0], pv.sa_p[v0], sc, N - K,
                                                    out.next_x + (int64_t)K * S + s,
                                                    out.next_y + (int64_t)K * S + s, S, nullptr, 0);
    for (int i = K + R.ng; i < N; i++) { out.next_x[(int64_t)i * S + s] = 0; out.next_y[(int64_t)i * S + s] = 0; }
    out.n_out[s] = K + R.ng;
    out.winner[s] = best;
}

template <bool kSlow>
__global__ __launch_bounds__(kWinBlock) void k_winner(MapG mg, pp_scene_batch in, pp_params P,
                                                      PrepV pv, pp_result out) {
    __shared__ __attribute__((aligned(16))) double wsm[5 * kWinKnots * kWinBlock];
    __shared__ int wmeta[4 * kWinBlock];
    const MapV m = map_view(mg.buf, mg.n);
    const int64_t S = in.n_scenes;
    const int D = P.n_draws > 1 ? P.n_draws : 1;
    const int64_t Sv = S * D;
    const int j = threadIdx.x;
    const int64_t s = (int64_t)blockIdx.x * kWinBlock + j;
    const int64_t v0 = s * D;                 // the nominal (draw 0) prep record
    if (s >= S || ((pv.lim_mask[v0] & kLimSlow) != 0) != kSlow) return;
    const int NS = P.n_speeds, Cv = NL * NS, C = D * Cv;
    // decision: first minimum over (lane, k) of the cost averaged over the draws (summed in draw
    // order, then / D; D = 1: the plain cost)
    int best = 0;
    double bc = 0;
    for (int c = 0; c < Cv; c++) {
        double sum = out.cost[s * C + c];
        for (int d = 1; d < D; d++) sum += out.cost[s * C + d * Cv + c];
        const double mean = sum / D;
        if (out.draw_mean_cost) out.draw_mean_cost[s * Cv + c] = mean;
        if (c == 0 || mean < bc) { bc = mean; best = c; }
    }
    // slot arrays interleaved by lane ([knot][lane]) so the 64 lanes' accesses spread over banks
    const Slot sl = {wsm + j, wsm + kWinKnots * kWinBlock + j, wsm + 2 * kWinKnots * kWinBlock + j,
                     wsm + 3 * kWinKnots * kWinBlock + j, wsm + 4 * kWinKnots * kWinBlock + j,
                     wmeta + j, kWinBlock, kWinBlock};
    setup_lane(m, P, in, pv, s, v0, Sv, best / NS, sl);
    winner_run<kSlow>(in, P, pv, out, s, v0, Sv, best, sl);
}

// Round 6: k_cand made the decision (out.winner) and stored the winner's spline slot (per scene
// kWinRec doubles: the knot-interleaved x, y, a, b, c of k_cand's LDS slot, then the 4 meta ints):
// no argmin, no spline build and no LDS here, so the block is 256 lanes and occupancy is the
// registers' (k_winner holds 38 KB of LDS per 64 lanes: one wave per SIMD). A segment reload reads
// one knot's 40 contiguous bytes, and the cache line holding them usually holds the next knot too.
template <bool kSlow>
__global__ __launch_bounds__(256) void k_winner_st(pp_scene_batch in, pp_params P, PrepV pv, pp_result out,
                                                   const double* wslot) {
    const int64_t S = in.n_scenes;
    const int D = P.n_draws > 1 ? P.n_draws : 1;
    const int64_t Sv = S * D;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t v0 = s * D;
    if (s >= S || ((pv.lim_mask[v0] & kLimSlow) != 0) != kSlow) return;
    double* b = const_cast<double*>(wslot) + s * kWinRec;
    const Slot sl = {b, b + 1, b + 2, b + 3, b + 4, (int*)(b + 5 * kWinKnots), 5, 1};
    winner_run<kSlow>(in, P, pv, out, s, v0, Sv, out.winner[s], sl);
}


// ------------------------------------------------------------------------------------------------
// K4 (reference mode): next_x/next_y of the winner from its recorded local path — the output
// transform of TrajectoryBuilder::build replayed exactly: at each recorded curvature adjustment
// the transform centre is rotated about the current point and the frame angle advanced
// (src/main.cpp:994-1007), every point is mapped back with the current frame (:1033-1037). One lane
// per scene; all loads/stores point-major (coalesced).
// ------------------------------------------------------------------------------------------------
// kChunk: recorded steps loaded together per lane (kEmitChunk for large batches; small batches,
// where the kernel is one serial chain of memory round trips per lane, load 16 steps at a time)
template <int kChunk>
__device__ __forceinline__ void emit_scene(const pp_scene_batch& in, const pp_params& P, const PrepV& pv,
                                           const pp_result& out, const double* rec, const uint64_t* adjm,
                                           int64_t s) {
    const int64_t S = in.n_scenes;
    const int N = P.n_points;
    const int K = pv.K[s];
    const int room = N - K;
    const int ng = out.n_out[s] - K;
    const int64_t rstride = (int64_t)room * S;
    {   // the kept previous points: every load issued before the first store
        double kx[PP_PREV_KEEP], ky[PP_PREV_KEEP];
#pragma unroll
        for (int i = 0; i < PP_PREV_KEEP; i++)
            if (i < K) { kx[i] = in.prev_x[(int64_t)i * S + s]; ky[i] = in.prev_y[(int64_t)i * S + s]; }
#pragma unroll
        for (int i = 0; i < PP_PREV_KEEP; i++)
            if (i < K) { PP_ST(out.next_x + (int64_t)i * S + s, kx[i]); PP_ST(out.next_y + (int64_t)i * S + s, ky[i]); }
    }
    OutFrame F = {pv.pos_x[s], pv.pos_y[s], pv.ca_p[s], pv.sa_p[s]};
    const uint64_t m0 = adjm[s], m1 = adjm[S + s];
    double pxp = 0, pyp = 0;                       // local position before the step
    // The adjusted steps are sparse and scattered over the wave's lanes, so the turn block runs,
    // with few lanes active, on most steps: it is kept short (frame_turn, turn_sincos). Steps are
    // taken kChunk at a time with all of the chunk's record loads (the turn angle only where the
    // step's bit is set) in flight together: one memory round trip per chunk instead of one or two
    // per step. A turn beyond sincos_pp's medium range (a step that slowed to ~1e-7 m/s) sends the
    // lane's chunk through a per-step loop with the library reduction, re-reading the record: the
    // unrolled chunk then holds no call and stays register-light.
    for (int g0 = 0; g0 < ng; g0 += kChunk) {
        double px_[kChunk], py_[kChunk], rt[kChunk];
        uint32_t bits = 0;
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int g = g0 + u;
            const bool bit = g < ng && ((g < 64 ? (m0 >> g) & 1 : (m1 >> (g - 64)) & 1) != 0);
            bits |= bit ? 1u << u : 0u;
#ifdef PP_CHECK
            if (g < ng) { PP_CHKP(rec_py((double*)rec, rstride, g, S, s), rec, nrec, 16); }
            if (bit) { PP_CHKP(rec_rot(rec, rstride, g, S, s), rec, nrec, 16); }
#endif
            px_[u] = 0.0; py_[u] = 0.0;
            if (g < ng) rec_ld(rec, rstride, g, S, s, px_[u], py_[u]);
            rt[u] = bit ? PP_LD(rec_rot(rec, rstride, g, S, s)) : 0.0;
        }
        bool huge = false;
#pragma unroll
        for (int u = 0; u < kChunk; u++) huge |= !(fabs(rt[u]) <= ppm::kMediumMax);
        if (__builtin_expect(huge, 0)) {
            for (int g = g0; g < ng && g < g0 + kChunk; g++) {
                if ((g < 64 ? (m0 >> g) & 1 : (m1 >> (g - 64)) & 1) != 0) {
                    double cr, sr;
                    turn_sincos<true>(*rec_rot(rec, rstride, g, S, s), sr, cr);
                    frame_turn(F, pxp, pyp, cr, sr);
                }
                double qx, qy, ox, oy;
                rec_ld(rec, rstride, g, S, s, qx, qy);
                frame_pt(F, qx, qy, ox, oy);
                out.next_x[(int64_t)(K + g) * S + s] = ox;
                out.next_y[(int64_t)(K + g) * S + s] = oy;
                pxp = qx;
                pyp = qy;
            }
            continue;
        }
        // sin/cos of the chunk's turns first (rt = 0 where no turn): independent of each other and
        // of the chain of turns below, so they overlap instead of queueing behind it
        double crs[kChunk], srs[kChunk];
        if (bits) {
#pragma unroll
            for (int u = 0; u < kChunk; u++) turn_sincos<false>(rt[u], srs[u], crs[u]);
        }
        // (not unrolled: the exits keep the compiler from it, as in emit_scene_rows below)
        for (int u = 0; u < kChunk; u++) {
            const int g = g0 + u;
            if (g >= ng) break;
            if ((bits >> u) & 1) frame_turn(F, pxp, pyp, crs[u], srs[u]);
            double ox, oy;
            frame_pt(F, px_[u], py_[u], ox, oy);
            if (!PP_CHKP(out.next_x + (int64_t)(K + g) * S + s, nx, nnext, 17)) break;
            PP_ST(out.next_x + (int64_t)(K + g) * S + s, ox);
            PP_ST(out.next_y + (int64_t)(K + g) * S + s, oy);
            pxp = px_[u];
            pyp = py_[u];
        }
    }
    for (int i = K + ng; i < N; i++) { out.next_x[(int64_t)i * S + s] = 0; out.next_y[(int64_t)i * S + s] = 0; }
}

// k_emit by output rows: the lane's loop runs over next_x/next_y's rows i = 0 .. N-1 (kept previous
// point i < K, generated point g = i - K < ng, zero after), so every store of the wave goes to one
// row (512 contiguous bytes), where stepping by g scatters each store over the rows K + g of the
// wave's lanes (K = 0 ... 9) and leaves every written line partial. The record loads are the ones
// scattered instead (rows g = i - K), read through the cache, where the wave's other lanes of the
// same line find them. Same operations in the same order per lane as emit_scene: bit-identical.
template <int kChunk>
__device__ __forceinline__ void emit_scene_rows(const pp_scene_batch& in, const pp_params& P, const PrepV& pv,
                                                const pp_result& out, const double* rec, const uint64_t* adjm,
                                                int64_t s) {
    const int64_t S = in.n_scenes;
    const int N = P.n_points;
    const int K = pv.K[s];
    const int room = N - K;
    const int ng = out.n_out[s] - K;
    const int64_t rstride = (int64_t)room * S;
    OutFrame F = {pv.pos_x[s], pv.pos_y[s], pv.ca_p[s], pv.sa_p[s]};
    const uint64_t m0 = adjm[s], m1 = adjm[S + s];
    double pxp = 0, pyp = 0;                       // local position before the step
    for (int i0 = 0; i0 < N; i0 += kChunk) {
        double px_[kChunk], py_[kChunk], rt[kChunk];
        uint32_t bits = 0, gen = 0;
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            const int i = i0 + u, g = i - K;
            const bool isg = i < N && g >= 0 && g < ng;
            const bool bit = isg && ((g < 64 ? (m0 >> g) & 1 : (m1 >> (g - 64)) & 1) != 0);
            bits |= bit ? 1u << u : 0u;
            gen |= isg ? 1u << u : 0u;
#ifdef PP_CHECK
            if (isg) { PP_CHKP(rec_py((double*)rec, rstride, g, S, s), rec, nrec, 16); }
            if (bit) { PP_CHKP(rec_rot(rec, rstride, g, S, s), rec, nrec, 16); }
#endif
            px_[u] = 0.0; py_[u] = 0.0;
            if (isg) {
                px_[u] = *rec_px((double*)rec, rstride, g, S, s);
                py_[u] = *rec_py((double*)rec, rstride, g, S, s);
            } else if (i < K) {
                px_[u] = in.prev_x[(int64_t)i * S + s];
                py_[u] = in.prev_y[(int64_t)i * S + s];
            }
            rt[u] = bit ? *rec_rot(rec, rstride, g, S, s) : 0.0;
        }
        bool huge = false;
#pragma unroll
        for (int u = 0; u < kChunk; u++) huge |= !(fabs(rt[u]) <= ppm::kMediumMax);
        if (__builtin_expect(huge, 0)) {
            // a turn beyond the medium range: the chunk step by step with the library reduction,
            // re-reading its inputs (the unrolled path below then holds no call)
            for (int i = i0; i < N && i < i0 + kChunk; i++) {
                const int g = i - K;
                double ox = 0.0, oy = 0.0;
                if (g >= 0 && g < ng) {
                    if ((g < 64 ? (m0 >> g) & 1 : (m1 >> (g - 64)) & 1) != 0) {
                        double cr, sr;
                        turn_sincos<true>(*rec_rot(rec, rstride, g, S, s), sr, cr);
                        frame_turn(F, pxp, pyp, cr, sr);
                    }
                    const double qx = *rec_px((double*)rec, rstride, g, S, s);
                    const double qy = *rec_py((double*)rec, rstride, g, S, s);
                    frame_pt(F, qx, qy, ox, oy);
                    pxp = qx;
                    pyp = qy;
                } else if (i < K) {
                    ox = in.prev_x[(int64_t)i * S + s];
                    oy = in.prev_y[(int64_t)i * S + s];
                }
                out.next_x[(int64_t)i * S + s] = ox;
                out.next_y[(int64_t)i * S + s] = oy;
            }
            continue;
        }
        double crs[kChunk], srs[kChunk];
        if (bits) {
#pragma unroll
            for (int u = 0; u < kChunk; u++) turn_sincos<false>(rt[u], srs[u], crs[u]);
        }
        // (a loop, not unrolled: its two exits keep the compiler from unrolling it, and the
        // unrolled form, written with guards instead of exits, measured 4 % slower: k_emit 0.79 ->
        // 0.82 ms at config 5, profiles/r04_ablations.txt)
        for (int u = 0; u < kChunk; u++) {
            const int i = i0 + u;
            if (i >= N) break;
            double ox = px_[u], oy = py_[u];
            if ((gen >> u) & 1) {
                if ((bits >> u) & 1) frame_turn(F, pxp, pyp, crs[u], srs[u]);
                frame_pt(F, px_[u], py_[u], ox, oy);
                pxp = px_[u];
                pyp = py_[u];
            }
            if (!PP_CHKP(out.next_x + (int64_t)i * S + s, nx, nnext, 17)) break;
            PP_ST(out.next_x + (int64_t)i * S + s, ox);
            PP_ST(out.next_y + (int64_t)i * S + s, oy);
        }
    }
}

// 4 waves per SIMD (128 VGPRs): the 262,144-scene shard's k_emit 0.108 -> 0.098 ms, the full
// config-5 batch unchanged (profiles/r03_ablations.txt)
constexpr int kEmitWaves = 4;
template <int kChunk>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kEmitWaves))) void k_emit(pp_scene_batch in, pp_params P, PrepV pv, pp_result out,
                                              const double* rec, const uint64_t* adjm, int64_t s0, int64_t s1) {
    const int64_t s = s0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // scenes [s0, s1)
    if (s >= s1 || s >= in.n_scenes) return;
    if (kChunk == kEmitRows) emit_scene_rows<kChunk>(in, P, pv, out, rec, adjm, s);
    else emit_scene<kChunk>(in, P, pv, out, rec, adjm, s);
}

// ------------------------------------------------------------------------------------------------
// K2 + K4 in one launch for small batches in reference mode (no paths), where the step is a chain
// of kernel latencies (BASELINE config 2: 4,096 scenes, ~1 wave per SIMD): the group's scenes in
// the proven range (k_cand<false>'s code), then its flagged scenes (k_cand<true>'s code; the
// group's bitmap bit is cleared as k_cand<true> clears it), then the lanes that recorded the
// winners' paths (tid < nsc, kMode 1) replay the output transform from their own stores
// (emit_scene). Two kernel boundaries fewer; waves_per_eu(1, 2): registers are not the limit here.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_cand_small(
        MapG mg, pp_scene_batch in, pp_params P, PrepV pv, pp_result out, int SPB, double* rec,
        uint64_t* adjm, uint32_t* gbits) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int64_t g = blockIdx.x;
    cand_group<false, 1, 1>(mg, in, P, pv, out, SPB, 1, rec, adjm, g, sm);
    __syncthreads();
    if ((gbits[g >> 5] >> (g & 31)) & 1u) {                   // same word for every lane
        cand_group<true, 1, 1>(mg, in, P, pv, out, SPB, 1, rec, adjm, g, sm);
        if (threadIdx.x == 0) atomicAnd(&gbits[g >> 5], ~(1u << (g & 31)));
    }
}

// ------------------------------------------------------------------------------------------------
// The whole step in one launch for small batches in reference mode (BASELINE config 2): K1 for the
// block's SPB (<= 16) scenes with 16 lanes each (prep_grp_eval<16>, the map staged in LDS once),
// a barrier, then k_cand_small's body (fast scenes, flagged scenes, the winners' replay), its
// phase A reading the same LDS map. The prep record goes through global memory inside the block
// (written, barrier, read by the same workgroup). No kernel boundary is left in the step.
// ------------------------------------------------------------------------------------------------
#ifndef PP_STEP_EMIT
#define PP_STEP_EMIT 2
#endif
// the winners' output in the one-launch step (cand_group kEmitIn): inline (2) or replayed (1)
constexpr int kStepEmit = PP_STEP_EMIT;
// the one-launch step with phase A beside K1 (wave_step_body) where the blocks allow it
#ifndef PP_STEP_WAVES
#define PP_STEP_WAVES 1
#endif
constexpr bool kStepWaves = PP_STEP_WAVES != 0;
// doubles of k_cand's LDS for SPB scenes (cand_geom_lds, host), rounded up
__host__ __device__ constexpr int cand_lds_doubles(int spb) {
    return (int)(((sizeof(double) * 5 * kKP * (NL * spb) + sizeof(int) * 4 * (NL * spb) + sizeof(uint32_t) * 2 * spb + 7) / 8 * 8 +
                  sizeof(uint64_t) * 2 * spb + sizeof(int) * spb + 7) / 8);
}
__device__ __forceinline__ void step_small_body(MapG mg, const pp_scene_batch& in, const pp_params& P,
                                                const PrepV& pv, const pp_result& out, int SPB, double* rec,
                                                uint64_t* adjm) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int n = mg.n;
#ifdef PP_TRACE
    // (block 0: start, after K1, after the fast scenes' K2 + K4, end; words at group kTraceK1 - 1;
    // the shader clock (s_memtime) beside the constant clock at start and end, group kTraceK1 - 3)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        trace_at(kTraceK1 - 1, 0);
        g_trace[8 * (kTraceK1 - 3) + 0] = wall_clock64();
        g_trace[8 * (kTraceK1 - 3) + 1] = clock64();
    }
#endif
    stage_map(sm, mg.buf, kMapArrays * n);
    __syncthreads();
    const MapV m = map_view(sm, n, mg.fastm);
    const int64_t g = blockIdx.x;
    {   // K1: scene g SPB + threadIdx.x / 16 by a group of 16 lanes
        const int q = (int)threadIdx.x / 16;
        const int64_t v = g * SPB + q;
        const GroupBits nobits = {nullptr, SPB, 1, nullptr, nullptr};
        if (q < SPB && v < in.n_scenes) prep_grp_eval<16>(m, in, P, pv, out.info, out.status, nobits, v, (int)threadIdx.x % 16);
    }
    __syncthreads();
#ifdef PP_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) trace_at(kTraceK1 - 1, 1);
#endif
    const MapG ml = {sm, n, mg.fastm};
    double* csm = sm + ((kMapArrays * n + 1) & ~1);
    cand_group<false, 1, kStepEmit>(ml, in, P, pv, out, SPB, 1, rec, adjm, g, csm);
    __syncthreads();
#ifdef PP_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) trace_at(kTraceK1 - 1, 2);
#endif
    cand_group<true, 1, kStepEmit>(ml, in, P, pv, out, SPB, 1, rec, adjm, g, csm);
#ifdef PP_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        trace_at(kTraceK1 - 1, 3);
        g_trace[8 * (kTraceK1 - 3) + 2] = wall_clock64();
        g_trace[8 * (kTraceK1 - 3) + 3] = clock64();
    }
#endif
}
// The one-launch step with phase A off the critical path (k_plan_frame, and k_step_small for blocks
// of up to kStepWaveSpb scenes): waves 0-1 run K1 (16 lanes per scene) while waves 2-3 derive each
// scene's ego state and the build's start pose themselves (K1's own functions on the same inputs:
// the same bits as K1's record) and build the scenes' NL spline slots — phase A needs neither the
// cars nor the planner. Wave 2 takes scenes 0-3, wave 3 scenes 4-7; each wave's steps synchronise
// by wave (one instruction stream; LDS is in order within a wave), the per-scene geometry passing
// through an LDS record of kGeoD doubles per scene.
constexpr int kStepWaveSpb = 8;
constexpr int kGeoD = 17;           // (the last: the heading)
static_assert(9 + NL <= kGeoD - 1, "geometry record");
#ifndef PP_POSE_BY_WAVE
#define PP_POSE_BY_WAVE 1
#endif
constexpr bool kPoseByWave = PP_POSE_BY_WAVE != 0;
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// wave w of the phase-A waves, lane l: scenes [4 w, 4 w + 4) of the block's nsc
__device__ __forceinline__ void wave_phase_a(const MapV& m, const pp_scene_batch& in, const pp_params& P,
                                             const PrepV& pv, int SPB, double* sm, double* geo, int64_t s0,
                                             int nsc, int w, int l) {
    const int64_t S = in.n_scenes;
    {   // the ego state, start pose and rotations of scene q by 16 lanes; lane 0 records them
        const int q = 4 * w + l / 16, r = l % 16;
        if (q < nsc) {                                // (group-uniform)
            const int64_t s = s0 + q;
            EgoSt e;
            prep_ego<16>(m, in, P, S, s, r, e);
            double pos_x, pos_y, angle;
            start_pose(in, S, s, e, pos_x, pos_y, angle);
            double tv[4];
            frame_trig<16>(angle, r, tv);
            const double ca_m = __shfl(tv[0], 0, 16), sa_m = __shfl(tv[1], 1, 16);
            // the prep record's pose and rotations (K1 skips them: GroupBits.pose_by_wave)
            double* const tdst[4] = {pv.ca_m, pv.sa_m, pv.ca_p, pv.sa_p};
#pragma unroll
            for (int t = 0; t < 4; t++)
                if (t == r) tdst[t][s] = tv[t];
            if (r == 0) { pv.pos_x[s] = pos_x; pv.pos_y[s] = pos_y; pv.angle[s] = angle; }
            if (r == 0) {
                double* gq = geo + q * kGeoD;
                gq[kGeoD - 1] = angle;
                gq[0] = e.K; gq[1] = pos_x; gq[2] = pos_y; gq[3] = ca_m; gq[4] = sa_m; gq[5] = e.ref_wp;
                gq[6] = e.ego_d; gq[7] = e.ego_speed; gq[8] = e.ego_vd;
#pragma unroll
                for (int k = 0; k < NL; k++) gq[9 + k] = e.ratio[k];
            }
        }
    }
    wave_sync();
    const int nslot = NL * SPB;
    double* sX = sm;
    int* sMeta = (int*)(sX + 5 * nslot * kKP);
    constexpr int kTS = 64 / (4 * NL) < 8 ? 64 / (4 * NL) : 8;
    const int jj = l / kTS, r = l - jj * kTS;         // this wave's slot jj (scene 4 w + jj / NL)
    const int q = 4 * w + jj / NL, L = jj % NL;
    const bool act = jj < 4 * NL && q < nsc;
    const int js = l, qs = 4 * w + js / NL;           // the serial steps: one lane per slot
    const bool act_s = js < 4 * NL && qs < nsc;
    auto geom = [&](int qq, int LL) {
        const double* gq = geo + qq * kGeoD;
        double ratio_L = gq[9];
#pragma unroll
        for (int k = 1; k < NL; k++) if (LL == k) ratio_L = gq[9 + k];
        return lane_geom_from((int)gq[0], gq[1], gq[2], gq[3], gq[4], (int)gq[5], ratio_L, gq[6], gq[7], gq[8], LL);
    };
    const Slot sl = lds_slot(sX, nslot, sMeta, act ? q * NL + L : 0);
    const Slot sls = lds_slot(sX, nslot, sMeta, act_s ? qs * NL + js % NL : 0);
    if (act) team_a1(m, in, geom(q, L), s0 + q, L, sl, r, kTS);
    wave_sync();
    if (act_s) team_a2(geom(qs, js % NL), sls);
    wave_sync();
    if (act) team_a3(sl, r, kTS);
    wave_sync();
    if (act_s) team_a4(sls);
    wave_sync();
    if (act) team_a5(sl, r, kTS);
}

// block g: scenes [g SPB, g SPB + nsc), SPB <= kThreads / 32: the first half of the block runs K1
// (16 lanes per scene), the second half phase A (4 scenes per wave)
template <int kThreads>
__device__ __forceinline__ void wave_step_body(MapG mg, const pp_scene_batch& in, const pp_params& P,
                                               const PrepV& pv, const pp_result& out, int SPB, double* rec,
                                               uint64_t* adjm, double* geo) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int n = mg.n;
    const int64_t g = blockIdx.x, s0 = g * SPB;
    const int nsc = (int)(in.n_scenes - s0 < SPB ? in.n_scenes - s0 : SPB);
#ifdef PP_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0) trace_at(kTraceK1 - 1, 0);
#endif
    stage_map(sm, mg.buf, kMapArrays * n);
    __syncthreads();
    const MapV m = map_view(sm, n, mg.fastm);
    double* csm = sm + ((kMapArrays * n + 1) & ~1);
    const int tid = (int)threadIdx.x;
    if (tid < kThreads / 2) {                     // K1: scene s0 + tid / 16 by 16 lanes
        const int q = tid / 16;
        const GroupBits nobits = {nullptr, SPB, 1, nullptr, nullptr, kPoseByWave ? 1 : 0};
        if (q < nsc) prep_grp_eval<16>(m, in, P, pv, out.info, out.status, nobits, s0 + q, tid % 16);
    } else {
        wave_phase_a(m, in, P, pv, SPB, csm, geo, s0, nsc, (tid - kThreads / 2) / 64, tid % 64);
#ifdef PP_TRACE
        if (blockIdx.x == 0 && tid == kThreads / 2) trace_at(kTraceK1 - 4, 0);
#endif
    }
    __syncthreads();
    // the heading's kLimSlow bit (recorded by the phase-A waves), before cand_group's first read
    // of lim_mask (behind its first barrier)
    if (kPoseByWave && tid < nsc && !(fabs(geo[tid * kGeoD + kGeoD - 1]) <= kSlowAngle))
        pv.lim_mask[s0 + tid] |= kLimSlow;
#ifdef PP_TRACE
    if (blockIdx.x == 0 && tid == 0) trace_at(kTraceK1 - 1, 1);
#endif
    const MapG ml = {sm, n, mg.fastm};
    cand_group<false, 1, kStepEmit, true>(ml, in, P, pv, out, SPB, 1, rec, adjm, g, csm);
    __syncthreads();
#ifdef PP_TRACE
    if (blockIdx.x == 0 && tid == 0) trace_at(kTraceK1 - 1, 2);
#endif
    cand_group<true, 1, kStepEmit>(ml, in, P, pv, out, SPB, 1, rec, adjm, g, csm);
#ifdef PP_TRACE
    if (blockIdx.x == 0 && tid == 0) trace_at(kTraceK1 - 1, 3);
#endif
}

// waves (host: step_waves_on): the block runs wave_step_body (SPB <= kStepWaveSpb, 256 threads, the
// geometry records in LDS after k_cand's)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_step_small(
        MapG mg, pp_scene_batch in, pp_params P, PrepV pv, pp_result out, int SPB, double* rec,
        uint64_t* adjm, int waves) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (waves) {                                  // (launch-uniform)
        double* geo = sm + ((kMapArrays * mg.n + 1) & ~1) + cand_lds_doubles(SPB);
        wave_step_body<256>(mg, in, P, pv, out, SPB, rec, adjm, geo);
    } else {
        step_small_body(mg, in, P, pv, out, SPB, rec, adjm);
    }
}

// 512 threads: blocks of 16 scenes, K1 on waves 0-3 beside phase A on waves 4-7 (BASELINE config 2:
// 256 such blocks, one per CU)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_step_small512(
        MapG mg, pp_scene_batch in, pp_params P, PrepV pv, pp_result out, int SPB, double* rec,
        uint64_t* adjm) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* geo = sm + ((kMapArrays * mg.n + 1) & ~1) + cand_lds_doubles(SPB);
    wave_step_body<512>(mg, in, P, pv, out, SPB, rec, adjm, geo);
}

// ------------------------------------------------------------------------------------------------
// pp_plan_frame in one launch: the frame's input ranges are read from pinned host memory into the
// device frame by the block itself, k_step_small's body runs, the output ranges are written back
// to pinned host memory, and a sequence number in host memory tells the waiting host thread the
// frame is done — no copy commands and no stream synchronisation per frame.
// Ranges are 16-byte-unit ranges of the frame (host and device share the layout; the host rounds
// each field's range out to whole units and merges neighbours): one 16-B load per unit, since
// the reads cross PCIe as one transaction per load.
// ------------------------------------------------------------------------------------------------
constexpr int kFioMax = 16;
constexpr int kFioInline = 176;   // 16-B units of input carried in the kernel arguments (2.75 KB)
struct FrameIO {
    const uint4* h_in;        // pinned host frame (inputs)
    uint4* d_frame;           // device frame
    uint4* h_out;             // pinned host frame (outputs)
    uint32_t* h_flag;         // pinned host word: seq once the outputs are in place
    uint32_t seq;
    int n_in, n_out;
    uint32_t in_off[kFioMax], in_len[kFioMax], out_off[kFioMax], out_len[kFioMax];   // 16-B units
    // inputs of up to kFioInline units (a frame of up to ~25 cars) ride in the kernel arguments,
    // which the launch writes to device memory: the block reads them there instead of across
    // PCIe (n_inl: the units held, in range order; 0: read the ranges from h_in)
    int n_inl;
    uint4 inl[kFioInline];
};
// units [0, total) of the ranges, thread t taking t, t + blockDim.x, ...: every thread's loads are
// issued before its stores (one round trip to the host per kChunk units)
template <int kChunk>
__device__ __forceinline__ void frame_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                           int nr, const uint32_t* off, const uint32_t* len) {
    uint32_t total = 0;
    for (int r = 0; r < nr; r++) total += len[r];
    for (uint32_t w0 = threadIdx.x; w0 < total; w0 += kChunk * blockDim.x) {
        uint4 v[kChunk];
        uint32_t at[kChunk];
#pragma unroll
        for (int u = 0; u < kChunk; u++) {
            uint32_t w = w0 + u * blockDim.x;
            at[u] = 0xffffffffu;
            if (w < total) {
                int r = 0;
                while (w >= len[r]) { w -= len[r]; r++; }
                at[u] = off[r] + w;
                v[u] = src[at[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < kChunk; u++)
            if (at[u] != 0xffffffffu) dst[at[u]] = v[u];
    }
}
// (io is the first kernel argument: offset 0 of the kernel-argument segment)
constexpr size_t kFioArgOff = 0;
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_plan_frame(
        FrameIO io, MapG mg, pp_scene_batch in, pp_params P, PrepV pv, pp_result out, int SPB, double* rec,
        uint64_t* adjm, int waves) {
#ifdef PP_FRAME_PROF
    const uint64_t t_in = wall_clock64();
#endif
    if (io.n_inl > 0) {
        // the kernel-argument copy: units in range order (thread t: units t, t + blockDim.x)
        const uint4* src = (const uint4*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + kFioArgOff +
                                          offsetof(FrameIO, inl));
        for (int w0 = (int)threadIdx.x; w0 < io.n_inl; w0 += (int)blockDim.x) {
            int w = w0, r = 0;
            while (w >= (int)io.in_len[r]) { w -= (int)io.in_len[r]; r++; }
            io.d_frame[io.in_off[r] + w] = src[w0];
        }
    } else {
        frame_copy<4>(io.h_in, io.d_frame, io.n_in, io.in_off, io.in_len);
    }
    __threadfence_block();
    __syncthreads();
#ifdef PP_FRAME_PROF
    const uint64_t t_body = wall_clock64();
#endif
    extern __shared__ __attribute__((aligned(16))) double sm[];
    if (waves) {
        double* geo = sm + ((kMapArrays * mg.n + 1) & ~1) + cand_lds_doubles(SPB);
        wave_step_body<256>(mg, in, P, pv, out, SPB, rec, adjm, geo);
    } else {
        step_small_body(mg, in, P, pv, out, SPB, rec, adjm);
    }
    __threadfence_block();
    __syncthreads();
#ifdef PP_FRAME_PROF
    const uint64_t t_out = wall_clock64();
#endif
    frame_copy<4>(io.d_frame, io.h_out, io.n_out, io.out_off, io.out_len);
#ifdef PP_FRAME_PROF
    if (threadIdx.x == 0) { io.h_flag[4] = (uint32_t)t_in; io.h_flag[5] = (uint32_t)t_body; io.h_flag[6] = (uint32_t)t_out; io.h_flag[7] = (uint32_t)wall_clock64(); }
#endif
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(io.h_flag, io.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------------------------------------
// closed-loop rollout: the simulator shim (include/pp.h pp_rollout). One lane per scene: log the
// frame, drive `consume` points of the plan, advance the traffic, report the cars in range.
// ------------------------------------------------------------------------------------------------
struct SimArgs {
    int consume;
    double range2;
    int frame;
    pp_rollout_log log;
};

__global__ __launch_bounds__(256) void k_sim(ppsynth::LaneTables LT, pp_scene_batch in,
                                             ppsynth::TrafficV tr, pp_params P, pp_result out, SimArgs A) {
    const int64_t S = in.n_scenes;
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const int N = P.n_points;
    const int n_out = out.n_out[s];
    const int T = out.winner[s] / P.n_speeds;
    double* ex = (double*)in.ego_x;
    double* ey = (double*)in.ego_y;
    double* eyaw = (double*)in.ego_yaw_deg;
    double* espd = (double*)in.ego_speed_mph;
    double* px = (double*)in.prev_x;
    double* py = (double*)in.prev_y;
    const double x0 = ex[s], y0 = ey[s];
    // frame record (the telemetry this frame was planned from + its plan)
    const int64_t fs = (int64_t)A.frame * S + s;
    if (A.log.ego_x) A.log.ego_x[fs] = x0;
    if (A.log.ego_y) A.log.ego_y[fs] = y0;
    if (A.log.ego_speed_mph) A.log.ego_speed_mph[fs] = espd[s];
    if (A.log.target_lane) A.log.target_lane[fs] = T;
    if (A.log.winner) A.log.winner[fs] = out.winner[s];
    if (A.log.n_out) A.log.n_out[fs] = n_out;
    if (A.log.status) A.log.status[fs] = out.status[s];
    if (A.log.n_cars) A.log.n_cars[fs] = in.n_cars[s];
    if (A.log.plan_x) {
        for (int i = 0; i < N; i++) {
            A.log.plan_x[((int64_t)A.frame * N + i) * S + s] = out.next_x[(int64_t)i * S + s];
            A.log.plan_y[((int64_t)A.frame * N + i) * S + s] = out.next_y[(int64_t)i * S + s];
        }
    }
    // ego: drive kk points; speed and yaw from the last driven step
    const int kk = n_out < A.consume ? n_out : A.consume;
    double nx = x0, ny = y0, qx = x0, qy = y0;
    if (kk >= 1) { nx = out.next_x[(int64_t)(kk - 1) * S + s]; ny = out.next_y[(int64_t)(kk - 1) * S + s]; }
    if (kk >= 2) { qx = out.next_x[(int64_t)(kk - 2) * S + s]; qy = out.next_y[(int64_t)(kk - 2) * S + s]; }
    const double dx = nx - qx, dy = ny - qy;
    const double dist = sqrt(dx * dx + dy * dy);
    ex[s] = nx; ey[s] = ny;
    espd[s] = dist * 50 * 2.237;
    if (dist > 0) eyaw[s] = ppg::atan2(dy, dx) * 180.0 / kPi;
    const int np = n_out - kk;
    for (int i = 0; i < PP_PREV_KEEP; i++) {
        const bool ok = i < np;
        px[(int64_t)i * S + s] = ok ? out.next_x[(int64_t)(kk + i) * S + s] : 0.0;
        py[(int64_t)i * S + s] = ok ? out.next_y[(int64_t)(kk + i) * S + s] : 0.0;
    }
    ((int32_t*)in.n_prev)[s] = np;
    ((int32_t*)in.prev_target_lane)[s] = T;
    // traffic: advance, then report the cars within range, ascending id
    int nc = 0;
    for (int j = 0; j < tr.n; j++) {
        const int64_t tx = (int64_t)j * S + s;
        const int lane = tr.lane[tx];
        int seg = tr.seg[tx];
        double t = tr.t[tx];
        const double v = tr.v[tx];
        ppsynth::lane_advance(LT, lane, &seg, &t, v * 0.02 * A.consume);
        tr.seg[tx] = seg; tr.t[tx] = t;
        double cx, cy, cvx, cvy;
        ppsynth::traffic_car(LT, lane, seg, t, tr.off[tx], v, &cx, &cy, &cvx, &cvy);
        const double rx = cx - nx, ry = cy - ny;
        if (rx * rx + ry * ry <= A.range2 && nc < in.car_stride) {
            const int64_t ix = (int64_t)nc * S + s;
            ((int32_t*)in.car_id)[ix] = j;
            ((double*)in.car_x)[ix] = cx; ((double*)in.car_y)[ix] = cy;
            ((double*)in.car_vx)[ix] = cvx; ((double*)in.car_vy)[ix] = cvy;
            nc++;
        }
    }
    ((int32_t*)in.n_cars)[s] = nc;
}

__global__ __launch_bounds__(256) void k_synth_traffic(ppsynth::LaneTables T, uint64_t seed, int64_t first,
                                                       ppsynth::OutBatch o, ppsynth::TrafficV tr, pp_scene_batch tb) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= o.S) return;
    ppsynth::synth_scene(T, seed, first + s, s, o, &tr);
    for (int j = 0; tb.tab_valid && j < tb.tab_slots; j++) {       // empty table, slot j = car j
        tb.tab_valid[(int64_t)j * o.S + s] = 0;
        if (tb.tab_id) tb.tab_id[(int64_t)j * o.S + s] = j;
    }
}

// ------------------------------------------------------------------------------------------------
// Map::Init on the device (src/main.cpp:89-131; pp_map_create_device). g: the MapG layout
// (kMapArrays n: ref x/y, normal x/y, lane centres x[NL]/y[NL], lane lengths[NL]); t: the synth
// lane tables (5 NL n). Three passes because each reads its neighbours' results of the previous one.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int wrap_i(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

__global__ __launch_bounds__(256) void k_map_normals(const double* wx, const double* wy, int n, double* g,
                                                     int* bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = wrap_i(i - 1, n);
    const double dx = wx[i] - wx[p], dy = wy[i] - wy[p];
    const double len = sqrt(dx * dx + dy * dy);
    if (!(len > 0)) atomicOr(bad, 1);                 // duplicate consecutive waypoints
    g[i] = wx[i]; g[n + i] = wy[i];
    g[2 * n + i] = dy / len;
    g[3 * n + i] = -dx / len;
}

__global__ __launch_bounds__(256) void k_map_lanes(int n, double* g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int q = wrap_i(i + 1, n);
    const double nx = g[2 * n + i], ny = g[3 * n + i];
    double ax = (nx + g[2 * n + q]) / 2, ay = (ny + g[3 * n + q]) / 2;
    // the host's std::atan2 / std::cos (glibc) restated bit for bit (pp_glibcm.h): the device map
    // equals pp_map_create's (|a_avg - a_n| < pi, inside the restated cos domain)
    const double a_n = ppg::atan2(ny, nx);
    const double a_avg = ppg::atan2(ay, ax);
    double c_;
    if (!ppg::cos(a_avg - a_n, c_)) c_ = __builtin_nan("");
    ax /= c_;
    ay /= c_;
    for (int r = 0; r < NL; r++) {
        const double off = 4.0 * (r + 0.5);
        g[(4 + r) * n + i] = g[i] + ax * off;
        g[(4 + NL + r) * n + i] = g[n + i] + ay * off;
    }
}

__global__ __launch_bounds__(256) void k_map_lengths(int n, double* g, double* t) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int p = wrap_i(i - 1, n);
    for (int r = 0; r < NL; r++) {
        const double lx = g[(4 + r) * n + i], ly = g[(4 + NL + r) * n + i];
        const double dx = lx - g[(4 + r) * n + p], dy = ly - g[(4 + NL + r) * n + p];
        const double len = sqrt(dx * dx + dy * dy);
        g[(4 + 2 * NL + r) * n + i] = len;                           // Map::get_lane_length
        const double den = dx * dx + dy * dy;                         // helpers.h:202 rdenom
        g[(4 + 3 * NL + r) * n + i] = den;
        g[(4 + 4 * NL + r) * n + i] = 1.0 / den;
        t[0 * NL * n + r * n + i] = lx;
        t[1 * NL * n + r * n + i] = ly;
        t[2 * NL * n + r * n + i] = len;
        t[3 * NL * n + r * n + i] = dx / len;
        t[4 * NL * n + r * n + i] = dy / len;
    }
}

// the restated libm on the device (pp_libm_eval; parity tests of pp_glibcm.h's device build)
__global__ __launch_bounds__(256) void k_libm(int kind, const double* a, const double* b, double* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r = __builtin_nan("");
    if (kind == 0) ppg::sin(a[i], r);
    else if (kind == 1) ppg::cos(a[i], r);
    else r = ppg::atan2(a[i], b[i]);
    out[i] = r;
}

// ------------------------------------------------------------------------------------------------
// scene synthesis
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_synth(ppsynth::LaneTables T, uint64_t seed, int64_t first,
                                               ppsynth::OutBatch o) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= o.S) return;
    ppsynth::synth_scene(T, seed, first + s, s, o);
}

// ================================================================================================
// host side: map, per-device state, C-ABI
// ================================================================================================
namespace {

constexpr int kMaxDev = 16;
constexpr int kMaxWaypoints = 1 << 24;
constexpr int kPrepD = 12 + 4 * NL;   // doubles per scene in PrepV (see prep_bind)
constexpr int kPrepI = 7;

// pp_eval's device workspaces, one set per HIP stream: evaluations on different streams never
// share intermediate buffers, and evaluations on one stream are ordered by it. A buffer is grown
// only after that stream has drained (it is the only stream using it).
// the split of shard-sized batches: parts (streams) per call, at most kSplitMax (split_parts)
constexpr int kSplitMax = 4;
// parts per call: a batch beyond kSplitMaxScenes runs as chunks of parts, part t on stream t % streams
// (split_chunks); each part has its own flagged-group count word and 4 timing-event slots
constexpr int kPartMax = 16;
#ifndef PP_SPLIT_PARTS
#define PP_SPLIT_PARTS 0      // 0: by batch size (split_parts); 2..4 forced (A/B builds)
#endif
struct StreamWS {
    void* ws = nullptr;           // prep workspace (per evaluation: scene x draw)
    int64_t ws_cap = 0;
    void* rec = nullptr;          // reference-mode winner record (per scene)
    int64_t rec_cap = 0;
    uint32_t* gbits = nullptr;    // k_cand groups holding a kLimSlow scene (bitmap; all zero between calls)
    int64_t gbits_cap = 0;        // words
    void* srt = nullptr;          // k_sort_cars' visit-major rows (SortedCars)
    size_t srt_cap = 0;           // bytes
    hipStream_t st2[kSplitMax - 1] = {};   // the split's other streams (shard-sized batches)
    hipEvent_t fork = nullptr, join[kSplitMax - 1] = {};
};
struct DevState {
    bool init = false;
    double* map = nullptr;        // kMapArrays * n
    uint2* wgrid = nullptr;       // the closest-waypoint cell table (pp_map::wgrid)
    double2* wseg = nullptr;      // reference segment lengths and reciprocals (pp_map::wseg)
    double* atab = nullptr;       // the approach table (pp_map::atab)
    double* lanetab = nullptr;    // synth tables: lc_x[NL n] lc_y[NL n] seg_len[NL n] tan_x[NL n] tan_y[NL n]
    std::map<void*, StreamWS> sws;  // per hip_stream
    void* frame = nullptr;        // single-frame scratch (pp_plan_frame)
    void* frame_host = nullptr;   // its pinned host staging copy (coherent: k_plan_frame reads and
                                  // writes it; the frame's done word follows the frame)
    hipStream_t frame_stream = nullptr;  // pp_plan_frame's stream
    uint32_t frame_seq = 0;       // the last frame's done word
    std::mutex frame_mu;          // one pp_plan_frame at a time per device (frame scratch + car table)
    void* stage = nullptr;        // pp_plan_batch_host staging buffer
    size_t stage_cap = 0;
    void* stage_host = nullptr;   // its pinned host mirror (one copy per direction and region)
    std::mutex stage_mu;          // one pp_plan_batch_host at a time per device
    pptab::CarTable plan_table;   // pp_plan_frame's persistent car table (the reference's std::map)
    int timing = 0;               // pp_timing_enable: 0 off, 1 every kernel, 2 K2 only
    std::vector<hipEvent_t> ev_pool;
    // groups of 4 kPartMax per pp_eval: before K1, after K1, after K2, after K3/K4 on the launch
    // stream (the split: those four per part, each part's on its own stream, events 4 h .. 4 h + 3)
    std::vector<hipEvent_t> ev_rec;
    // per group: bit 0 K3/K4 launched, bits 1-3 the split's parts (0: none), bit 4 K2's events only,
    // bit 5 no K1 kernel (the one-launch step)
    std::vector<int> ev_kind;
};

}  // namespace

struct pp_map {
    int n = 0;
    std::vector<double> geom;     // kMapArrays * n (MapG layout)
    std::vector<double> ptab;     // (4 + 2 NL) * n: ref xy, normal, lane centres (pp_map_geometry)
    std::vector<double> lanetab;  // 5 NL * n
    int fastm = 0;                // MapV::fastm: bit 1: every lane segment's rdenom in [2^-500, 2^500]; bit 2: approach_seg's map bounds
    std::vector<uint2> wgrid;     // closest-waypoint cell table (build_wgrid; empty: none)
    std::vector<double2> wseg;    // reference segment lengths and reciprocals (build_wseg; empty: none)
    std::vector<double> atab;     // lane matching's approach table (build_atab; empty: none)
    WGrid wg;                     // its geometry (cells: the device copy, set per device)
    DevState dev[kMaxDev];
    std::mutex mu;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d) { if (hipGetDevice(&prev) != hipSuccess) prev = -1; (void)hipSetDevice(d); }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// pp_map_geometry's table from the MapG layout: per waypoint ref xy, normal, lane centres
void fill_ptab(pp_map* M) {
    const int n = M->n;
    const double* g = M->geom.data();
    M->ptab.assign((4 + 2 * NL) * (size_t)n, 0.0);
    for (int i = 0; i < n; i++) {
        double* o = &M->ptab[(4 + 2 * NL) * (size_t)i];
        o[0] = g[i]; o[1] = g[n + i]; o[2] = g[2 * n + i]; o[3] = g[3 * n + i];
        for (int r = 0; r < NL; r++) { o[4 + 2 * r] = g[(4 + r) * n + i]; o[5 + 2 * r] = g[(4 + NL + r) * n + i]; }
    }
    M->fastm = 1;
    for (size_t i = (size_t)(4 + 3 * NL) * n; i < (size_t)(4 + 4 * NL) * n; i++)
        if (!(g[i] >= 0x1p-500 && g[i] <= 0x1p500)) M->fastm = 0;
    // bit 2 (lane matching's approach runs, pp_device.h approach_seg): every lane segment's rdenom
    // >= 1 m^2 and every lane centre within 4e4 m of the origin
    bool appr = M->fastm != 0;
    for (size_t i = (size_t)(4 + 3 * NL) * n; i < (size_t)(4 + 4 * NL) * n; i++) appr = appr && g[i] >= 1.0;
    for (size_t i = (size_t)4 * n; i < (size_t)(4 + 2 * NL) * n; i++) appr = appr && std::fabs(g[i]) < 4e4;
    if (appr) M->fastm |= 2;
}

// The closest-waypoint cell table (pp_device.h WGrid, init_reference_waypoint). Cells of 16 m
// within 32 m of the waypoint polyline get a list: waypoint w can be the closest one to a point of
// cell B only if its distance to B, dmin(w, B), is at most U = min over all waypoints of the
// largest distance from w' to B (the closest waypoint of any point of B is at most U away). B is
// grown by 0.5 m on each side (the kernel's cell index rounds), and the test carries a relative
// margin of 1e-6 (the kernel's squared distances round by a few ulps): the list holds every
// waypoint that can be the scan's answer. Lists of up to 4 (the highway map's cells near the road
// hold 1-4); a cell with more, or away from the road, has none (0xFFFFFFFF: the kernel scans).
// Maps of more than 65,535 waypoints, or whose table would take more than 5e7 distance tests to
// build, get no table.
constexpr double kWgridMaxCells = 4e6;
void build_wgrid(pp_map* M) {
    constexpr double kCell = 16.0, kNear = 32.0, kGrow = 0.5;
    const int n = M->n;
    M->wgrid.clear();
    M->wg = WGrid{};
    if (n < 1 || n > 65535) return;
    const double* rx = M->geom.data();
    const double* ry = rx + n;
    double x0 = rx[0], x1 = rx[0], y0 = ry[0], y1 = ry[0];
    for (int i = 0; i < n; i++) {
        if (!std::isfinite(rx[i]) || !std::isfinite(ry[i])) return;
        x0 = std::min(x0, rx[i]); x1 = std::max(x1, rx[i]); y0 = std::min(y0, ry[i]); y1 = std::max(y1, ry[i]);
    }
    const double gx0 = x0 - 2 * kNear, gy0 = y0 - 2 * kNear;
    const double wdt = x1 - x0 + 4 * kNear, hgt = y1 - y0 + 4 * kNear;
    if (!(wdt / kCell < 1e5 && hgt / kCell < 1e5)) return;
    const int gnx = (int)std::ceil(wdt / kCell), gny = (int)std::ceil(hgt / kCell);
    // at most 4e6 cells (a 32 km square; 32 MB on the host and the device): a map spread wider
    // keeps the full scan (two waypoints 1,000 km apart would ask for ~4e9 cells)
    if ((double)gnx * (double)gny > kWgridMaxCells) return;
    // cells near the polyline: sample every segment every 2 m, mark cells within kNear
    std::vector<uint8_t> near((size_t)gnx * gny, 0);
    const int R = (int)std::ceil(kNear / kCell);
    for (int i = 0; i < n; i++) {
        const int j = (i + 1) % n;
        const double len = std::hypot(rx[j] - rx[i], ry[j] - ry[i]);
        const int ns = std::max(1, (int)std::ceil(len / 2.0));
        for (int k = 0; k <= ns; k++) {
            const double t = (double)k / ns;
            const double px = rx[i] + (rx[j] - rx[i]) * t, py = ry[i] + (ry[j] - ry[i]) * t;
            const int ci = (int)((px - gx0) / kCell), cj = (int)((py - gy0) / kCell);
            for (int dj = -R; dj <= R; dj++)
                for (int di = -R; di <= R; di++) {
                    const int a = ci + di, b = cj + dj;
                    if (a >= 0 && b >= 0 && a < gnx && b < gny) near[(size_t)b * gnx + a] = 1;
                }
        }
    }
    size_t nnear = 0;
    for (uint8_t v : near) nnear += v;
    if ((double)nnear * n > 5e7) return;
    std::vector<uint2> cells((size_t)gnx * gny, uint2{0xFFFFFFFFu, 0xFFFFFFFFu});
    std::vector<int> cand;
    for (int cj = 0; cj < gny; cj++)
        for (int ci = 0; ci < gnx; ci++) {
            if (!near[(size_t)cj * gnx + ci]) continue;
            const double bx0 = gx0 + ci * kCell - kGrow, bx1 = gx0 + (ci + 1) * kCell + kGrow;
            const double by0 = gy0 + cj * kCell - kGrow, by1 = gy0 + (cj + 1) * kCell + kGrow;
            double U = INFINITY;
            for (int i = 0; i < n; i++) {
                const double fx = std::max(std::fabs(rx[i] - bx0), std::fabs(rx[i] - bx1));
                const double fy = std::max(std::fabs(ry[i] - by0), std::fabs(ry[i] - by1));
                U = std::min(U, fx * fx + fy * fy);
            }
            const double lim = U * (1 + 1e-6) + 1e-6;
            cand.clear();
            for (int i = 0; i < n && cand.size() <= 4; i++) {
                const double dx = std::max({bx0 - rx[i], rx[i] - bx1, 0.0});
                const double dy = std::max({by0 - ry[i], ry[i] - by1, 0.0});
                if (dx * dx + dy * dy <= lim) cand.push_back(i);
            }
            if (cand.empty() || cand.size() > 4) continue;
            while (cand.size() < 4) cand.push_back(cand.back());
            cells[(size_t)cj * gnx + ci] = uint2{(uint32_t)cand[0] | ((uint32_t)cand[1] << 16),
                                                 (uint32_t)cand[2] | ((uint32_t)cand[3] << 16)};
        }
    M->wgrid.swap(cells);
    M->wg.gx0 = gx0; M->wg.gy0 = gy0; M->wg.ginv = 1.0 / kCell; M->wg.gnx = gnx; M->wg.gny = gny;
}

// Map::project_speed's segment length (src/main.cpp:332-339: w = ref_b - ref_{b-1}, |w| =
// sqrt(wx^2 + wy^2), the same operations as the kernel, unfused, correctly rounded sqrt) and
// RN(1 / |w|) by IEEE division, per segment b (project_speed then divides by the reciprocal with one
// Markstein correction: the correctly rounded quotient, ppd::div_by_rcp). Only for maps whose
// lengths all lie in [2^-500, 2^500] (div_by_rcp's divisor range); else none.
void build_wseg(pp_map* M) {
    const int n = M->n;
    M->wseg.clear();
    const double* rx = M->geom.data();
    const double* ry = rx + n;
    std::vector<double2> t(n);
    for (int b = 0; b < n; b++) {
        const int a = (int)(((int64_t)b - 1 + n) % n);
        const double wx = rx[b] - rx[a], wy = ry[b] - ry[a];
        const double wvl = std::sqrt(wx * wx + wy * wy);
        if (!(wvl >= 0x1p-500 && wvl <= 0x1p500)) return;
        t[b] = double2{wvl, 1.0 / wvl};
    }
    M->wseg.swap(t);
}

// Lane matching's approach table (pp_device.h approach_cert): per lane segment b (waypoint b - 1 to
// b) and lane l, d = RN(pb - pa) (the walk's own differences), c = pa.d, and the certain test's
// constants c + rdenom + kAtabMargin (forward) and c - 1 - kAtabMargin (backward), rdenom the map's
// own table value. Only for maps with fastm bit 2 (the bounds its margin argument needs).
void build_atab(pp_map* M) {
    M->atab.clear();
    if (!(M->fastm & 2)) return;
    const int n = M->n;
    const double* g = M->geom.data();
    const double* lcx = g + 4 * (size_t)n;
    const double* lcy = g + (4 + NL) * (size_t)n;
    const double* llen = g + (4 + 2 * NL) * (size_t)n;
    const double* lden = g + (4 + 3 * NL) * (size_t)n;
    std::vector<double> t((size_t)kAtabD * n, 0.0);
    for (int b = 0; b < n; b++) {
        const int a = b == 0 ? n - 1 : b - 1;
        double* r = &t[(size_t)kAtabD * b];
        for (int l = 0; l < NL; l++) {
            const double pax = lcx[(size_t)l * n + a], pay = lcy[(size_t)l * n + a];
            const double dx = lcx[(size_t)l * n + b] - pax, dy = lcy[(size_t)l * n + b] - pay;
            const double c = pax * dx + pay * dy;
            r[2 * l] = dx;
            r[2 * l + 1] = dy;
            r[2 * NL + l] = c + lden[(size_t)l * n + b] + kAtabMargin;
            r[3 * NL + l] = c - 1.0 - kAtabMargin;
            r[4 * NL + l] = llen[(size_t)l * n + b];
        }
    }
    M->atab.swap(t);
}

// The optional per-map tables (cell table, segment reciprocals, approach table) speed K1 up and
// never change a result: a map whose tables cannot be built (an allocation failure included) runs
// without them. Nothing here throws across the C-ABI.
void build_tables(pp_map* M) {
    try { build_wgrid(M); } catch (...) { M->wgrid.clear(); M->wgrid.shrink_to_fit(); M->wg = WGrid{}; }
    try { build_wseg(M); } catch (...) { M->wseg.clear(); M->wseg.shrink_to_fit(); }
    try { build_atab(M); } catch (...) { M->atab.clear(); M->atab.shrink_to_fit(); }
}

void free_map_tables(DevState& D) {
    if (D.wgrid) (void)hipFree(D.wgrid);
    if (D.wseg) (void)hipFree(D.wseg);
    if (D.atab) (void)hipFree(D.atab);
    D.wgrid = nullptr; D.wseg = nullptr; D.atab = nullptr;
}

// the device copies of the cell table, the segment table and the approach table (dev_init,
// pp_map_create_device)
int upload_wgrid(pp_map* M, DevState& D) {
    if (!M->wgrid.empty()) {
        if (hipMalloc(&D.wgrid, sizeof(uint2) * M->wgrid.size()) != hipSuccess) return PP_ERR_NOMEM;
        if (hipMemcpy(D.wgrid, M->wgrid.data(), sizeof(uint2) * M->wgrid.size(), hipMemcpyHostToDevice) != hipSuccess)
            return PP_ERR_HIP;
    }
    if (!M->wseg.empty()) {
        if (hipMalloc(&D.wseg, sizeof(double2) * M->wseg.size()) != hipSuccess) return PP_ERR_NOMEM;
        if (hipMemcpy(D.wseg, M->wseg.data(), sizeof(double2) * M->wseg.size(), hipMemcpyHostToDevice) != hipSuccess)
            return PP_ERR_HIP;
    }
    if (!M->atab.empty()) {
        if (hipMalloc(&D.atab, sizeof(double) * M->atab.size()) != hipSuccess) return PP_ERR_NOMEM;
        if (hipMemcpy(D.atab, M->atab.data(), sizeof(double) * M->atab.size(), hipMemcpyHostToDevice) != hipSuccess)
            return PP_ERR_HIP;
    }
    return PP_OK;
}

// Map::Init (src/main.cpp:89-131) + derived tables, on the host (done once per map).
int build_map(pp_map* M, const double* wx, const double* wy, int n) {
    M->n = n;
    std::vector<double> nx(n), ny(n), lcx(NL * n), lcy(NL * n);
    auto W = [n](int i) { return (int)(((int64_t)i + n) % n); };
    for (int i = 0; i < n; i++) {
        const int p = W(i - 1);
        const double dx = wx[i] - wx[p], dy = wy[i] - wy[p];
        const double len = std::sqrt(dx * dx + dy * dy);
        if (!(len > 0)) return PP_ERR_ARG;    // duplicate consecutive waypoints: Map::Init divides by 0
        nx[i] = dy / len;
        ny[i] = -dx / len;
    }
    for (int i = 0; i < n; i++) {
        const int q = W(i + 1);
        double ax = (nx[i] + nx[q]) / 2, ay = (ny[i] + ny[q]) / 2;
        const double a_n = std::atan2(ny[i], nx[i]);
        const double a_avg = std::atan2(ay, ax);
        const double cos_alpha = std::cos(a_avg - a_n);
        ax /= cos_alpha;
        ay /= cos_alpha;
        for (int r = 0; r < NL; r++) {
            const double off = 4.0 * (r + 0.5);
            lcx[r * n + i] = wx[i] + ax * off;
            lcy[r * n + i] = wy[i] + ay * off;
        }
    }
    M->geom.assign(kMapArrays * (size_t)n, 0.0);
    double* g = M->geom.data();
    for (int i = 0; i < n; i++) {
        g[i] = wx[i]; g[n + i] = wy[i]; g[2 * n + i] = nx[i]; g[3 * n + i] = ny[i];
        for (int r = 0; r < NL; r++) {
            g[(4 + r) * n + i] = lcx[r * n + i];
            g[(4 + NL + r) * n + i] = lcy[r * n + i];
            const int p = W(i - 1);
            const double dx = lcx[r * n + i] - lcx[r * n + p], dy = lcy[r * n + i] - lcy[r * n + p];
            g[(4 + 2 * NL + r) * n + i] = std::sqrt(dx * dx + dy * dy);    // Map::get_lane_length
            const double ex = lcx[r * n + p] - lcx[r * n + i], ey = lcy[r * n + p] - lcy[r * n + i];
            const double den = ex * ex + ey * ey;                           // helpers.h:202 rdenom
            g[(4 + 3 * NL + r) * n + i] = den;
            g[(4 + 4 * NL + r) * n + i] = 1.0 / den;
        }
    }
    fill_ptab(M);
    build_tables(M);
    M->lanetab.assign(5 * NL * (size_t)n, 0.0);
    double* t = M->lanetab.data();
    for (int r = 0; r < NL; r++)
        for (int i = 0; i < n; i++) {
            const double len = g[(4 + 2 * NL + r) * n + i];
            const int p = W(i - 1);
            t[0 * NL * n + r * n + i] = lcx[r * n + i];
            t[1 * NL * n + r * n + i] = lcy[r * n + i];
            t[2 * NL * n + r * n + i] = len;
            t[3 * NL * n + r * n + i] = (lcx[r * n + i] - lcx[r * n + p]) / len;
            t[4 * NL * n + r * n + i] = (lcy[r * n + i] - lcy[r * n + p]) / len;
        }
    return PP_OK;
}

ppsynth::OutBatch out_batch(const pp_scene_batch* b) {
    ppsynth::OutBatch o;
    o.S = b->n_scenes;
    o.ego_x = (double*)b->ego_x; o.ego_y = (double*)b->ego_y;
    o.ego_yaw_deg = (double*)b->ego_yaw_deg; o.ego_speed_mph = (double*)b->ego_speed_mph;
    o.prev_x = (double*)b->prev_x; o.prev_y = (double*)b->prev_y;
    o.n_prev = (int32_t*)b->n_prev; o.prev_target_lane = (int32_t*)b->prev_target_lane;
    o.n_cars = (int32_t*)b->n_cars; o.car_id = (int32_t*)b->car_id;
    o.car_x = (double*)b->car_x; o.car_y = (double*)b->car_y;
    o.car_vx = (double*)b->car_vx; o.car_vy = (double*)b->car_vy;
    return o;
}

bool traffic_ok(const pp_traffic* t, const pp_scene_batch* b) {
    return t && b && t->n_cars >= 0 && t->n_cars <= PP_MAX_CARS && t->lane && t->seg && t->t &&
           t->offset && t->speed;
}

ppsynth::TrafficV traffic_view(const pp_traffic* t, int64_t S) {
    ppsynth::TrafficV v;
    v.S = S; v.n = t->n_cars; v.lane = t->lane; v.seg = t->seg; v.t = t->t; v.off = t->offset; v.v = t->speed;
    return v;
}

ppsynth::LaneTables lane_tables(const double* t, int n) {
    ppsynth::LaneTables T;
    T.n = n; T.lc_x = t; T.lc_y = t + NL * n; T.seg_len = t + 2 * NL * n; T.tan_x = t + 3 * NL * n;
    T.tan_y = t + 4 * NL * n;
    return T;
}

int dev_init(pp_map* M, int device) {
    DevState& D = M->dev[device];
    if (D.init) return PP_OK;
    if (hipMalloc(&D.map, sizeof(double) * M->geom.size()) != hipSuccess) return PP_ERR_NOMEM;
    if (hipMalloc(&D.lanetab, sizeof(double) * M->lanetab.size()) != hipSuccess) return PP_ERR_NOMEM;
    if (hipMemcpy(D.map, M->geom.data(), sizeof(double) * M->geom.size(), hipMemcpyHostToDevice) != hipSuccess) return PP_ERR_HIP;
    if (hipMemcpy(D.lanetab, M->lanetab.data(), sizeof(double) * M->lanetab.size(), hipMemcpyHostToDevice) != hipSuccess) return PP_ERR_HIP;
    const int rc = upload_wgrid(M, D);
    if (rc != PP_OK) return rc;
    D.init = true;
    return PP_OK;
}

size_t prep_bytes(int64_t S) { return ((size_t)S * (kPrepD * 8 + kPrepI * 4) + 255) / 256 * 256; }
// reference-mode winner record (k_cand -> k_emit): 3 x PP_MAX_POINTS x S doubles + 2 x S u64
size_t rec_bytes(int64_t S) { return (size_t)S * (3 * PP_MAX_POINTS + 2) * 8 + 256; }
static_assert(kWinRec <= 3 * PP_MAX_POINTS + 2, "the stored winner slots share the record's memory");
double* rec_buf(void* rec) { return (double*)rec; }
uint64_t* adj_buf(void* rec, int64_t cap) { return (uint64_t*)((double*)rec + 3 * PP_MAX_POINTS * cap); }


PrepV prep_bind(void* base, int64_t S) {
    PrepV p;
    double* d = (double*)base;
    double** dd[] = {&p.pos_x, &p.pos_y, &p.angle, &p.ca_m, &p.sa_m, &p.ca_p, &p.sa_p,
                     &p.ego_speed, &p.ego_d, &p.ego_vd, &p.in_ts, &p.in_tt};
    int k = 0;
    for (double** q : dd) *q = d + (int64_t)(k++) * S;
    p.ratio = d + (int64_t)(k) * S; k += NL;
    p.l_ts = d + (int64_t)(k) * S; k += NL;
    p.l_tt = d + (int64_t)(k) * S; k += NL;
    p.score = d + (int64_t)(k) * S; k += NL;
    // k == kPrepD
    int32_t* ip = (int32_t*)(d + (int64_t)kPrepD * S);
    int32_t** ii[] = {&p.K, &p.ref_wp, &p.T, &p.ego_lane, &p.open_mask, &p.lim_mask, &p.status};
    int m = 0;
    for (int32_t** q : ii) *q = ip + (int64_t)(m++) * S;
    return p;
}

// pp_debug_set's switches (include/pp.h PP_DBG_*): launch-shape overrides for tests and A/B
// measurements. Every one defaults to 0 = the product's own choice; nothing reads the environment.
std::atomic<int> g_dbg[PP_DBG_KEYS];
int dbg(int key) { return g_dbg[key].load(std::memory_order_relaxed); }

// K4 inside k_cand: the winners' sin/cos tables (2 N doubles each) fit the block's spline slots
bool emit_in_ok(int N) { return 2 * N <= 5 * NL * kKP; }
// small reference-mode batches (<= kFusedSmall scenes): K2 + K4 in one launch (k_cand_small) or the
// whole step in one launch (k_step_small); PP_DBG_SHAPE forces one of the three shapes
constexpr int64_t kFusedSmall = 16384;
bool fused_small(int64_t S) {
    const int f = dbg(PP_DBG_SHAPE);
    return f ? f != PP_SHAPE_SPLIT : S <= kFusedSmall;
}
bool step_fused_on() { return dbg(PP_DBG_SHAPE) != PP_SHAPE_CAND_SMALL; }
// Two-stream split (reference mode, no paths): batches of about one 8-GPU shard of BASELINE config 5
// (262,144 scenes) run as two halves, each K1 -> K2 -> K4 on its own stream, so one half's kernels
// fill the other's start-up and tail (a batch this size is ~15 rounds of k_cand blocks and one of
// k_prep waves). Up to config 5's N = 2 shard (1,048,576 scenes: 4.96-4.99 ms against
// 5.09-5.15 unsplit, same boxes); the full 2,097,152-scene batch stays one stream (9.87-9.91 against
// 9.93-9.96 ms split, within the boxes' spread, and its K2 span is 0.3 ms longer than the unsplit
// K2). PP_DBG_SPLIT 1 forces it for every batch the split can take (reference mode without paths
// or draws, one K1 lane per scene: more than 65,536 scenes, prep_group), 2 turns it off; the parts
// of the last call are read back with PP_DBG_LAST_PARTS.
constexpr int64_t kSplitMin = 131072, kSplitMaxScenes = 1572864;
#ifndef PP_SPLIT_BIG
#define PP_SPLIT_BIG 0        // 1: batches beyond kSplitMaxScenes run as chunks (A/B builds)
#endif
constexpr int64_t kChunkScenes = 1048576;
bool split_on(int64_t S) {
    const int f = dbg(PP_DBG_SPLIT);
    if (f == 2) return false;
    // forced: any batch of at least 2,048 scenes (its parts then never come out empty)
    if (f == 1) return S >= 2048;
    return S >= kSplitMin && (S <= kSplitMaxScenes || PP_SPLIT_BIG);
}
// parts of a split batch: 2 up to 393,216 scenes (BASELINE config 5's N = 8 shard, 262,144: 1.32 ms
// against 1.35 / 1.37 ms with 3 / 4 parts), 3 beyond (its N = 4 shard, 524,288: 2.52 ms against
// 2.59-2.62 with 2 parts and 2.60 unsplit; profiles/r04_ablations.txt)
int split_parts(int64_t S) {
    if (PP_SPLIT_PARTS >= 2 && PP_SPLIT_PARTS <= kSplitMax) return PP_SPLIT_PARTS;
    return S > 393216 ? 3 : 2;
}
// chunks of a split batch: a batch beyond kSplitMaxScenes, when split (PP_DBG_SPLIT 1, or
// PP_SPLIT_BIG builds), runs as ceil(S / 1,048,576) sequential chunks of split_parts parts each
// (chunk c + 1 starts when every part of chunk c has ended). Round 6 measured it for BASELINE
// config 5 (2,097,152 scenes; tools/chunk_probe.py, profiles/r06_chunk_probe*.txt): two separate
// pp_eval calls of 1,048,576 scenes (their own arrays) ran 9.78-9.87 ms against 9.79-9.99 for
// one call on one stream, but the same chunks inside one call (the batch's own arrays) ran
// 9.98-10.01 on the box where the separate calls took 9.85, and 6 parts pipelined over the 3
// streams without the join 10.00-10.07: the full batch stays on one stream.
int split_chunks(int64_t S) {
    if (S <= kSplitMaxScenes) return 1;
    const int64_t c = (S + kChunkScenes - 1) / kChunkScenes;
    return (int)std::min<int64_t>(c, kPartMax / kSplitMax);
}
// K1 (one lane per evaluation): 3 waves per SIMD, or 4 where the batch's waves fill whole rounds of
// 4 better. Round 5 (the approach table in the 3-wave build's LDS): a round of 3 waves per SIMD
// takes ~0.150 ms (config 5: 1.65 ms for 32,768 waves = 11 rounds), one of 4 ~0.357 ms (spills,
// the table in global memory); 262,144 scenes = 4,096 waves: 0.297 ms at 3, 0.357 at 4
// (profiles/r05_ablations.txt), so the 4-wave build no longer wins at any size (round 4: 0.188 /
// 0.286 ms per round, 4 waves at 262,144). PP_DBG_PREP_WAVES forces 3 or 4.
int cu_count(int device) {
    static int cus[kMaxDev] = {};
    if (device < 0 || device >= kMaxDev) return 256;
    if (cus[device] == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c <= 0) c = 256;
        cus[device] = c;
    }
    return cus[device];
}
// the one-launch step with phase A beside K1 (wave_step_body) where its blocks fit one per CU:
// 8-scene blocks of 256 threads (the frame, batches up to 2,048 scenes: 0.128 -> 0.116 ms at 2,048),
// else 16-scene blocks of 512 threads; beyond, 16-scene blocks of 256 threads, K1 then phase A
// (2 blocks of 8 per CU measured slower: config 2 0.132 against 0.128 ms, profiles/r04_ablations.txt)
int step_waves_on(int64_t S, int spb, int device) {
    if (!kStepWaves) return 0;
    if ((S + kStepWaveSpb - 1) / kStepWaveSpb <= cu_count(device)) return 1;
    if (spb >= 16 && (S + 15) / 16 <= cu_count(device)) return 2;
    return 0;
}
bool prep_w4(int64_t Sv, int device) {
    const int f = dbg(PP_DBG_PREP_WAVES);
    if (f == 3 || f == 4) return f == 4;
    const int64_t waves = (Sv + 63) / 64, simds = 4LL * cu_count(device);
    const int64_t r3 = (waves + 3 * simds - 1) / (3 * simds), r4 = (waves + 4 * simds - 1) / (4 * simds);
    return 357 * r4 < 150 * r3;
}
// k_emit: batches up to this many scenes take the small-batch instantiation
constexpr int64_t kEmitSmall = 65536;
// K1 lanes per evaluation: the largest power of two <= 16 that keeps Sv * G within ~2 waves per
// SIMD of the chip (256 CUs x 4 SIMDs x 64 lanes x 2); 1 for large batches. PP_DBG_PREP_GROUP
// forces a value.
bool prep_group_ok(int G) { return G == 0 || G == 1 || G == 2 || G == 4 || G == 8 || G == 16; }
int prep_group(int64_t Sv) {
    const int forced = dbg(PP_DBG_PREP_GROUP);
    if (forced > 0) return forced;
    const int64_t target = 256LL * 4 * 64 * 2;
    int G = 1;
    while (G < 16 && Sv * G * 2 <= target) G *= 2;
    return G;
}

// Scenes per k_cand group (C <= 256): at most 256 / C (one 256-lane block) and 64 / NL (spline
// slots: phase A's serial steps run on one wave), chosen so the block's waves carry the fewest
// idle lanes through phase B (largest such count on ties): C = 15 -> 17 scenes (255 of 256
// lanes), C = 24 (config 3) -> 8 scenes in exactly 3 waves instead of 10 in 4 waves with 16 idle
// lanes.
int cands_per_block(int C) {
    int hi = 256 / C;
    if (hi > 64 / NL) hi = 64 / NL;
    if (hi < 1) return 1;
    int best = hi;
    double bu = 0;
    for (int spb = hi; spb >= 1; spb--) {
        const int t = spb * C;
        const double u = (double)t / (double)(((t + 63) / 64) * 64);
        if (u > bu + 1e-9) { bu = u; best = spb; }
    }
    return best;
}

// callers hold M->mu; `st` is the stream the workspace belongs to
int ensure_ws(StreamWS& W, hipStream_t st, int64_t Sv) {
    if (W.ws_cap >= Sv) return PP_OK;
    if (W.ws) { (void)hipStreamSynchronize(st); (void)hipFree(W.ws); W.ws = nullptr; W.ws_cap = 0; }
    if (hipMalloc(&W.ws, prep_bytes(Sv)) != hipSuccess) return PP_ERR_NOMEM;
    W.ws_cap = Sv;
    return PP_OK;
}

// k_sort_cars' output for S scenes of `rows` rows each (SortedCars over one allocation)
size_t srt_bytes(int64_t S, int rows) { return (size_t)S * ((size_t)rows * (4 * sizeof(double) + sizeof(int)) + 8) + 256; }
int ensure_srt(StreamWS& W, hipStream_t st, int64_t S, int rows, SortedCars& sc) {
    const size_t need = srt_bytes(S, rows);
    if (W.srt_cap < need) {
        if (W.srt) { (void)hipStreamSynchronize(st); (void)hipFree(W.srt); W.srt = nullptr; W.srt_cap = 0; }
        if (hipMalloc(&W.srt, need) != hipSuccess) return PP_ERR_NOMEM;
        W.srt_cap = need;
    }
    double* b = (double*)W.srt;
    const int64_t n = (int64_t)rows * S;
    sc.x = b; sc.y = b + n; sc.vx = b + 2 * n; sc.vy = b + 3 * n;
    sc.id = (int*)(b + 4 * n);
    sc.order = (uint64_t*)(((uintptr_t)(sc.id + n) + 7) & ~(uintptr_t)7);
    sc.rows = rows;
    return PP_OK;
}

int ensure_rec(StreamWS& W, hipStream_t st, int64_t S) {
    const int64_t cap = (S + 63) & ~(int64_t)63;   // whole 64-scene blocks
    if (W.rec_cap >= cap) return PP_OK;
    if (W.rec) { (void)hipStreamSynchronize(st); (void)hipFree(W.rec); W.rec = nullptr; W.rec_cap = 0; }
    if (hipMalloc(&W.rec, rec_bytes(cap)) != hipSuccess) return PP_ERR_NOMEM;
    W.rec_cap = cap;
    return PP_OK;
}

// The slow-group bitmap (words), then the flagged-group count and list (ngroups entries), in one
// allocation: [cap words][count][list: 32 cap entries]
int ensure_gbits(StreamWS& W, hipStream_t st, int64_t ngroups) {
    const int64_t words = (ngroups + 31) / 32;
    if (W.gbits_cap >= words) return PP_OK;
    if (W.gbits) { (void)hipStreamSynchronize(st); (void)hipFree(W.gbits); W.gbits = nullptr; W.gbits_cap = 0; }
    const int64_t cap = std::max<int64_t>(words, 1024);
    // [bits: cap words][flagged-group count][the split's second-half count][list: 32 cap entries]
    const size_t bytes = sizeof(uint32_t) * (size_t)(cap + kPartMax + 32 * cap);
    if (hipMalloc(&W.gbits, bytes) != hipSuccess) return PP_ERR_NOMEM;
    if (hipMemsetAsync(W.gbits, 0, bytes, st) != hipSuccess) return PP_ERR_HIP;
    W.gbits_cap = cap;
    return PP_OK;
}

void free_ws(StreamWS& W) {
    for (int k = 0; k < kSplitMax - 1; k++) {
        if (W.st2[k]) (void)hipStreamDestroy(W.st2[k]);
        if (W.join[k]) (void)hipEventDestroy(W.join[k]);
    }
    if (W.fork) (void)hipEventDestroy(W.fork);
    if (W.ws) (void)hipFree(W.ws);
    if (W.rec) (void)hipFree(W.rec);
    if (W.gbits) (void)hipFree(W.gbits);
    if (W.srt) (void)hipFree(W.srt);
    W = StreamWS();
}

// k_cand's launch geometry for C candidates per scene (BPS == 1: SPB scenes per group; else one
// scene over BPS groups of 256 candidates)
struct CandGeom { int spb, bps, threads; size_t lds; int64_t groups; };
// k_cand's LDS for SPB scenes per group: slots (5 x kKP doubles + 4 ints each), sFlags/sSlow,
// then (8-aligned) sAdj and sNg
size_t cand_geom_lds(int spb) {
    const int nslot = NL * spb;
    size_t lds = sizeof(double) * 5 * kKP * (size_t)nslot + sizeof(int) * 4 * nslot + sizeof(uint32_t) * 2 * spb;
    return ((lds + 7) & ~(size_t)7) + sizeof(uint64_t) * 2 * spb + sizeof(int) * spb;
}
// the flat geometry for the all-paths mode (kMode 2): 256-lane groups over the batch's candidates,
// scenes straddling two groups (their spline slots built in both, status flags merged with
// atomics): four full waves per block where whole scenes would leave a wave slot of the CU idle
// (C = 24: 8 scenes in 3 waves, 5 blocks = 15 of 16 waves per CU). Up to (C + 254) / C + 1 scenes
// per group; C >= 13 keeps those slots within the first wave (NL SPB <= 64 for phase A's serial steps)
#ifndef PP_CAND_FLAT
#define PP_CAND_FLAT 1
#endif
bool cand_flat_ok(int C) { return PP_CAND_FLAT && C >= 13 && C <= 128 && 256 % C != 0; }
CandGeom cand_geom(int C, int64_t S, bool flat = false) {
    CandGeom g;
    if (flat) {
        g.spb = (C + 254) / C + 1;
        g.bps = -1;
        g.threads = 256;
        g.lds = cand_geom_lds(g.spb);
        g.groups = (S * C + 255) / 256;
        return g;
    }
    g.spb = C <= 256 ? cands_per_block(C) : 1;
    g.bps = C <= 256 ? 1 : (C + 255) / 256;
    g.threads = C <= 256 ? ((g.spb * C + 63) / 64) * 64 : 256;
    g.lds = cand_geom_lds(g.spb);
    g.groups = g.bps == 1 ? (S + g.spb - 1) / g.spb : S * g.bps;
    return g;
}

int n_draws(const pp_params* p) { return p->n_draws > 1 ? p->n_draws : 1; }

// k_prep<true, false>'s LDS with the approach table after the map (MapG::atab_lds)
size_t prep_lds_atab(int n) {
    return sizeof(double) * (((kMapArrays * (size_t)n + 1) & ~(size_t)1) + kAtabD * (size_t)n);
}


bool params_ok(const pp_params* p) {
    return p && p->n_points > PP_PREV_KEEP && p->n_points <= PP_MAX_POINTS && p->n_speeds >= 1 &&
           p->n_speeds <= PP_MAX_SPEEDS && NL * p->n_speeds <= 256 &&
           (p->cost_mode == PP_COST_REFERENCE || p->cost_mode == PP_COST_COMFORT) &&
           p->n_draws >= 0 && p->n_draws <= PP_MAX_DRAWS && p->noise_first_scene >= 0 &&
           !(p->n_draws > 1 && p->emit_paths);
}

}  // namespace

extern "C" {

void pp_params_default(pp_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->n_points = 50;
    p->n_speeds = 5;
    p->cost_mode = PP_COST_REFERENCE;
    p->emit_paths = 0;
    const double offs[4] = {-4.0, -2.0, 0.0, 2.0};      // SURVEY.md §8(d) speed grid
    for (int i = 0; i < 4; i++) p->speed_offsets[i] = offs[i];
    p->relaxed_acc = 5;                  // src/main.cpp:39-49
    p->min_relaxed_acc_while_braking = 4;
    p->maximum_acc = 8;
    p->max_speed = 22.2;
    p->car_length = 4.5;
    p->safety_distance = 2;
    p->keep_distance = 10;
    p->keep_distance_leeway = 0.5;
    p->n_draws = 0;
    p->noise_seed = 0x5EED0002ull;
    p->noise_first_scene = 0;
    p->noise_pos_sigma = 0.5;            // SURVEY.md §8(d) Monte-Carlo
    p->noise_vel_sigma = 0.5;
}

int32_t pp_num_candidates(const pp_params* p) { return p ? n_draws(p) * NL * p->n_speeds : 0; }

int32_t pp_num_lanes(void) { return NL; }

int32_t pp_max_cars(void) { return PP_MAX_CARS; }

double pp_mc_gauss(uint64_t seed, int64_t scene, int32_t draw, int32_t car, int32_t q) {
    return ppsynth::mc_gauss(seed, (uint64_t)scene, draw, car, q);
}

#ifdef PP_CHECK
int32_t pp_check_read(unsigned long long* out, int32_t reset) {  // checking builds only: g_chk[8]
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#ifdef PP_TRACE
int32_t pp_trace_read(unsigned long long* out, int64_t words) {   // diagnostic builds only: g_trace
    if (words > 8LL * kTraceMax) words = 8LL * kTraceMax;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(unsigned long long) * words) != hipSuccess) return -1;
    return 0;
}
#endif
#if defined(PP_DIAG) || defined(PP_LIMCENSUS)
int32_t pp_diag_read(unsigned long long* out, int32_t reset) {   // diagnostic builds only (96 words)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * kDiagWords) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[kDiagWords] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
int32_t pp_libm_eval(int32_t kind, const double* a, const double* b, double* out, int64_t n,
                     int32_t device, void* hip_stream) {
    if (kind < 0 || kind > 2 || n < 0 || (n > 0 && (!a || !out || (kind == 2 && !b))) || device < -1 ||
        device >= kMaxDev)
        return PP_ERR_ARG;
    if (n == 0) return PP_OK;
    if (device < 0) {
        for (int64_t i = 0; i < n; i++) {
            double r = __builtin_nan("");
            if (kind == 0) ppg::sin(a[i], r);
            else if (kind == 1) ppg::cos(a[i], r);
            else r = ppg::atan2(a[i], b[i]);
            out[i] = r;
        }
        return PP_OK;
    }
    DeviceGuard g(device);
    const int64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffff) return PP_ERR_ARG;
    hipLaunchKernelGGL(k_libm, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hip_stream, kind, a, b, out, n);
    return hipGetLastError() == hipSuccess ? PP_OK : PP_ERR_HIP;
}

const char* pp_version(void) { return "pp-mi355x 0.1 (gfx950, fp64, lane-per-candidate)"; }

int32_t pp_map_create(const double* wx, const double* wy, int32_t n, pp_map** out) {
    if (!wx || !wy || !out || n < 3 || n > kMaxWaypoints) return PP_ERR_ARG;
    pp_map* M = new (std::nothrow) pp_map();
    if (!M) return PP_ERR_NOMEM;
    int rc;
    try { rc = build_map(M, wx, wy, n); } catch (...) { rc = PP_ERR_NOMEM; }   // (host allocations)
    if (rc != PP_OK) { delete M; return rc; }
    *out = M;
    return PP_OK;
}

// Map::Init on the device from device waypoint arrays; the derived tables are mirrored to the host
// (for pp_map_geometry, the host generator and other devices).
static int32_t map_create_device(const double* d_wx, const double* d_wy, int32_t n, int32_t device,
                                 void* hip_stream, pp_map** out);
int32_t pp_map_create_device(const double* d_wx, const double* d_wy, int32_t n, int32_t device, void* hip_stream,
                             pp_map** out) {
    try { return map_create_device(d_wx, d_wy, n, device, hip_stream, out); } catch (...) { return PP_ERR_NOMEM; }
}
static int32_t map_create_device(const double* d_wx, const double* d_wy, int32_t n, int32_t device,
                                 void* hip_stream, pp_map** out) {
    if (!d_wx || !d_wy || !out || n < 3 || n > kMaxWaypoints || device < 0 || device >= kMaxDev) return PP_ERR_ARG;
    pp_map* M = new (std::nothrow) pp_map();
    if (!M) return PP_ERR_NOMEM;
    M->n = n;
    DeviceGuard g(device);
    DevState& D = M->dev[device];
    hipStream_t st = (hipStream_t)hip_stream;
    int* bad = nullptr;
    if (hipMalloc(&D.map, sizeof(double) * kMapArrays * (size_t)n) != hipSuccess ||
        hipMalloc(&D.lanetab, sizeof(double) * 5 * NL * (size_t)n) != hipSuccess || hipMalloc(&bad, sizeof(int)) != hipSuccess) {
        if (D.map) (void)hipFree(D.map);
        if (D.lanetab) (void)hipFree(D.lanetab);
        delete M;
        return PP_ERR_NOMEM;
    }
    int rc = PP_OK;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    if (hipMemsetAsync(bad, 0, sizeof(int), st) != hipSuccess) rc = PP_ERR_HIP;
    hipLaunchKernelGGL(k_map_normals, dim3(blocks), dim3(256), 0, st, d_wx, d_wy, n, D.map, bad);
    hipLaunchKernelGGL(k_map_lanes, dim3(blocks), dim3(256), 0, st, n, D.map);
    hipLaunchKernelGGL(k_map_lengths, dim3(blocks), dim3(256), 0, st, n, D.map, D.lanetab);
    if (hipGetLastError() != hipSuccess) rc = PP_ERR_HIP;
    int hbad = 0;
    M->geom.assign(kMapArrays * (size_t)n, 0.0);
    M->lanetab.assign(5 * NL * (size_t)n, 0.0);
    if (rc == PP_OK && (hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipMemcpyAsync(M->geom.data(), D.map, sizeof(double) * kMapArrays * (size_t)n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipMemcpyAsync(M->lanetab.data(), D.lanetab, sizeof(double) * 5 * NL * (size_t)n, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipStreamSynchronize(st) != hipSuccess))
        rc = PP_ERR_HIP;
    (void)hipFree(bad);
    if (rc == PP_OK && hbad) rc = PP_ERR_ARG;          // Map::Init divides by a zero segment length
    if (rc != PP_OK) {
        (void)hipFree(D.map); (void)hipFree(D.lanetab);
        D.map = D.lanetab = nullptr;
        delete M;
        return rc;
    }
    fill_ptab(M);
    build_tables(M);
    if (upload_wgrid(M, D) != PP_OK) {
        free_map_tables(D);
        (void)hipFree(D.map); (void)hipFree(D.lanetab);
        delete M;
        return PP_ERR_NOMEM;
    }
    D.init = true;
    *out = M;
    return PP_OK;
}

int32_t pp_map_destroy(pp_map* M) {
    if (!M) return PP_ERR_ARG;
    for (int d = 0; d < kMaxDev; d++) {
        DevState& D = M->dev[d];
        if (!D.init) continue;
        DeviceGuard g(d);
        (void)hipDeviceSynchronize();
        (void)hipFree(D.map); (void)hipFree(D.lanetab);
        free_map_tables(D);
        for (auto& kv : D.sws) free_ws(kv.second);
        D.sws.clear();
        if (D.frame) (void)hipFree(D.frame);
        if (D.frame_host) (void)hipHostFree(D.frame_host);
        if (D.frame_stream) (void)hipStreamDestroy(D.frame_stream);
        if (D.stage) (void)hipFree(D.stage);
        if (D.stage_host) (void)hipHostFree(D.stage_host);
        for (hipEvent_t e : D.ev_pool) (void)hipEventDestroy(e);
        for (hipEvent_t e : D.ev_rec) (void)hipEventDestroy(e);
    }
    delete M;
    return PP_OK;
}

int32_t pp_map_geometry(const pp_map* M, double* out, int32_t n) {
    if (!M || !out || n != M->n) return PP_ERR_ARG;
    memcpy(out, M->ptab.data(), sizeof(double) * (4 + 2 * NL) * (size_t)n);
    return PP_OK;
}

int32_t pp_reserve(pp_map* M, int32_t device, int64_t max_scenes) {
    if (!M || device < 0 || device >= kMaxDev || max_scenes < 0) return PP_ERR_ARG;
    std::lock_guard<std::mutex> lk(M->mu);
    DeviceGuard g(device);
    int rc = dev_init(M, device);
    if (rc) return rc;
    StreamWS& W = M->dev[device].sws[nullptr];       // the null stream's workspace
    rc = ensure_ws(W, nullptr, max_scenes);
    if (rc) return rc;
    return ensure_rec(W, nullptr, max_scenes);
}

}  // extern "C"
namespace {
// pp_eval; fio (pp_plan_frame): the single-launch frame kernel with host-memory staging, where the
// call takes the fused one-launch shape (PP_ERR_STATE otherwise: the caller stages by copies)
int32_t eval_impl(pp_map* M, const pp_scene_batch* in, const pp_params* prm, pp_result* out,
                  int32_t device, void* hip_stream, const FrameIO* fio) {
    if (!M || !in || !out || !params_ok(prm) || device < 0 || device >= kMaxDev) return PP_ERR_ARG;
    if (in->n_scenes < 0 || in->car_stride < 0 || in->car_stride > PP_MAX_CARS) return PP_ERR_ARG;
    if (in->n_scenes == 0) return PP_OK;
    if (!in->ego_x || !in->ego_y || !in->ego_yaw_deg || !in->ego_speed_mph || !in->prev_x ||
        !in->prev_y || !in->n_prev || !in->prev_target_lane || !in->n_cars ||
        (in->car_stride > 0 && (!in->car_id || !in->car_x || !in->car_y || !in->car_vx || !in->car_vy)))
        return PP_ERR_ARG;
    if (!out->winner || !out->n_out || !out->next_x || !out->next_y || !out->cost || !out->status)
        return PP_ERR_ARG;
    if (prm->emit_paths && !out->paths) return PP_ERR_ARG;
    if (in->tab_valid && (!in->tab_lane || !in->tab_s || !in->tab_d || !in->tab_vs || !in->tab_vd ||
                          !in->tab_vx || !in->tab_vy || prm->n_draws > 1 || in->tab_slots < 0 ||
                          in->tab_slots > PP_MAX_CARS))
        return PP_ERR_ARG;
    DeviceGuard g(device);
    hipStream_t st = (hipStream_t)hip_stream;
    const int64_t S = in->n_scenes;
    const int Dn = n_draws(prm);
    const int64_t Sv = S * Dn;                    // evaluations (scene x draw)
    // reference decision without draws: the winner is known before the loop (k_cand records it,
    // k_emit writes it); otherwise the decision is a cost argmin (k_winner)
    const bool ref_direct = prm->cost_mode == PP_COST_REFERENCE && Dn == 1;
    const int Cn_ = Dn * NL * prm->n_speeds;
    const CandGeom cg = cand_geom(Cn_, S, prm->emit_paths && Dn == 1 && cand_flat_ok(Cn_));
    if (cg.groups > 0x7fffffff) return PP_ERR_ARG;
    // small batches in reference mode without paths: K2 and K4 in one launch (k_cand_small, K4 in
    // the block: emit_in), unless the horizon's sin/cos table (2 N doubles per winner) exceeds the
    // block's spline slots. Large batches keep K4 in its own kernel: in the block, the serial
    // replay holds the block's LDS and costs k_cand more than k_emit takes.
    const bool fused = ref_direct && !prm->emit_paths && cg.bps == 1 && emit_in_ok(prm->n_points) &&
                       fused_small(S);
    const bool emit_in = fused;
    // small reference-mode batches with the map in LDS: the whole step in one launch (k_step_small)
    // (kStepWaves: blocks of up to kStepWaveSpb scenes in 256 threads, K1 and phase A side by side,
    // plus the per-scene geometry records; otherwise up to 16 scenes, K1 then phase A)
    // step_waves: 1 blocks of 8 scenes in 256 threads, 2 blocks of 16 scenes in 512 threads, 0 the
    // 16-scene blocks without the split
    int step_waves = step_waves_on(S, cg.spb, device);
    const size_t map_lds = sizeof(double) * (size_t)((kMapArrays * M->n + 1) & ~1);
    auto step_lds = [&](int wv, int spb) {
        return map_lds + (wv != 0 ? sizeof(double) * (size_t)(cand_lds_doubles(spb) + kGeoD * spb) : cand_geom_lds(spb));
    };
    if (step_waves && step_lds(step_waves, std::min(cg.spb, step_waves == 1 ? kStepWaveSpb : 16)) > 65536) step_waves = 0;
    const int spb_f = std::min(cg.spb, step_waves == 1 ? kStepWaveSpb : 256 / 16);
    const int64_t groups_f = (S + spb_f - 1) / spb_f;
    const size_t lds_f = step_lds(step_waves, spb_f);
    const bool step_fused = fused && M->n <= kLdsMapMax && lds_f <= 65536 && step_fused_on();
    if (fio && (!step_fused || groups_f != 1)) return PP_ERR_STATE;
    // the map lock is held from workspace binding through the (asynchronous) launches: a
    // concurrent call cannot grow and free this stream's buffers in between
    std::lock_guard<std::mutex> lk(M->mu);
    int rc = dev_init(M, device);
    if (rc) return rc;
    DevState& DS = M->dev[device];
    StreamWS& W = DS.sws[hip_stream];
    rc = ensure_ws(W, st, Sv);
    if (rc) return rc;
    rc = ensure_gbits(W, st, cg.groups);
    if (rc) return rc;
    double* rec = nullptr;
    uint64_t* adjm = nullptr;
    if (ref_direct && !prm->emit_paths) {
        rc = ensure_rec(W, st, S);
        if (rc) return rc;
        rec = rec_buf(W.rec);
        adjm = adj_buf(W.rec, W.rec_cap);
    }
    // comfort mode without paths or draws, every scene's candidates in one block: k_cand makes the
    // decision and stores the winner's spline slot in the record's memory (616 B per scene of its
    // 3,088), k_winner_st re-runs the winner from it
    double* wslot = nullptr;
    // K0 (k_sort_cars) ahead of the one-lane K1: no car table, fewer than PP_SORT_DMAX draws, at
    // most 16 rows per scene (k_prep's own sorting rule; larger tables keep the identity order)
    SortedCars srt = {};
    const int k0f = dbg(PP_DBG_SORT_CARS);
    if ((k0f == 1 || (k0f == 0 && PP_SORT_K0)) && !in->tab_valid && Dn < PP_SORT_DMAX && in->car_stride >= 2 &&
        in->car_stride <= 16 && prep_group(Sv) == 1) {
        rc = ensure_srt(W, st, S, in->car_stride, srt);
        if (rc) return rc;
    }
    size_t cand_lds = cg.lds;
    if (PP_WSLOT && !ref_direct && !prm->emit_paths && cg.bps == 1 && Dn == 1) {
        rc = ensure_rec(W, st, S);
        if (rc) return rc;
        wslot = rec_buf(W.rec);
        cand_lds = ((cg.lds + 7) & ~(size_t)7) + sizeof(double) * 256;     // + sCost
    }
    if (dbg(PP_DBG_POISON)) {
        // every call starts from NaN-filled (0xFF) intermediates and outputs, so no kernel can lean
        // on what an earlier call left there (or on an output element it never writes); the
        // slow-group bitmap must be all zero between calls (k_cand<true> clears what k_prep set)
        auto fill = [&](void* p, size_t bytes) { return !p || !bytes || hipMemsetAsync(p, 0xFF, bytes, st) == hipSuccess; };
        const int64_t Cn = (int64_t)Dn * NL * prm->n_speeds, N = prm->n_points;
        const int64_t words = (cg.groups + 31) / 32;
        std::vector<uint32_t> hb((size_t)words);
        if (hipMemcpyAsync(hb.data(), W.gbits, sizeof(uint32_t) * words, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return PP_ERR_HIP;
        for (uint32_t w : hb)
            if (w) return PP_ERR_STATE;
        const bool ok = fill(W.ws, prep_bytes(W.ws_cap)) &&
                        fill(W.rec, W.rec ? rec_bytes(W.rec_cap) : 0) &&
                        fill(W.srt, W.srt ? W.srt_cap : 0) &&
                        fill(W.gbits + W.gbits_cap + kPartMax, sizeof(uint32_t) * 32 * (size_t)W.gbits_cap) &&
                        fill(out->winner, 4 * S) && fill(out->n_out, 4 * S) && fill(out->status, 4 * S) &&
                        fill(out->next_x, 8 * N * S) && fill(out->next_y, 8 * N * S) &&
                        fill(out->cost, 8 * Cn * S) && fill(out->info, sizeof(pp_scene_info) * S) &&
                        fill(out->draw_mean_cost, Dn > 1 ? 8 * NL * prm->n_speeds * S : 0) &&
                        fill(prm->emit_paths ? out->paths : nullptr, 16 * N * Cn * S) &&
                        fill(prm->emit_paths ? out->path_len : nullptr, 4 * Cn * S);
        if (!ok) return PP_ERR_HIP;
    }
    const PrepV pv = prep_bind(W.ws, W.ws_cap);
    MapG mg;
    mg.buf = DS.map;
    mg.n = M->n;
    mg.fastm = M->fastm;
    mg.wg = M->wg;
    mg.wg.cells = DS.wgrid;
    mg.wseg = DS.wseg;
    mg.atab = DS.atab;
    // k_prep<true, false> stages the approach table after the map where both fit a block's 64 KB
    mg.atab_lds = DS.atab && sizeof(double) * (((kMapArrays * (size_t)M->n + 1) & ~(size_t)1) + kAtabD * (size_t)M->n) <= 65536;
    // tall: events at every kernel boundary; tk2: at K2's (PP_TIMING_K2 records only those two).
    // The call's record is a group of 4 kPartMax slots (before K1, after K1, after K2, after
    // K3/K4, per part); a slot takes an event from the pool when it is first recorded, so a
    // K2-only call takes 2 events (2 per part when split) and an all-kernel call 4 per part
    const bool timing = DS.timing != 0, tall = DS.timing == 1, tk2 = timing;
    const size_t ev_base = DS.ev_rec.size();
    if (timing) {
        DS.ev_rec.resize(ev_base + 4 * kPartMax, nullptr);
        DS.ev_kind.push_back((!(ref_direct && prm->emit_paths) && !emit_in ? 1 : 0) | (tall ? 0 : 16));
    }
    auto ev = [&](int i) -> hipEvent_t {
        hipEvent_t& e = DS.ev_rec[ev_base + i];
        if (!e) {
            if (DS.ev_pool.empty() && hipEventCreate(&e) != hipSuccess) return nullptr;
            if (!e) { e = DS.ev_pool.back(); DS.ev_pool.pop_back(); }
        }
        return e;
    };
    pp_params P = *prm;
    pp_scene_batch B = *in;
    pp_result R = *out;
    if (!P.emit_paths) { R.paths = nullptr; R.path_len = nullptr; }
    GroupBits gb = {};
    gb.bits = W.gbits; gb.SPB = cg.spb; gb.BPS = cg.bps; gb.C = Cn_;
    gb.count = W.gbits + W.gbits_cap;
    gb.list = gb.count + kPartMax;
#ifdef PP_CHECK
    {   // checking builds: the bounds of every buffer this call's kernels store into
        ChkLim L = {};
        const long long Cn = (long long)Dn * NL * P.n_speeds;
        L.paths = R.paths; L.npaths = R.paths ? (long long)S * P.n_points * Cn * 2 : 0;
        L.nx = R.next_x; L.ny = R.next_y; L.nnext = (long long)S * P.n_points;
        L.rec = rec; L.nrec = rec ? 3LL * PP_MAX_POINTS * W.rec_cap : 0;
        L.adjm = (const unsigned long long*)adjm; L.nadj = adjm ? 2LL * W.rec_cap : 0;
        L.cost = R.cost; L.ncost = (long long)S * Cn; L.nscen = S;
        if (hipStreamSynchronize(st) != hipSuccess ||
            hipMemcpyToSymbol(HIP_SYMBOL(g_lim), &L, sizeof L) != hipSuccess) return PP_ERR_HIP;
    }
#endif
    if (step_fused) {
        if (timing) DS.ev_kind.back() |= 32;          // (no K1 kernel: K1 runs inside the step)
        if (tall) (void)hipEventRecord(ev(0), st);
        // K1 takes 16 lanes for each of the block's spb_f scenes, K2 spb_f x C lanes: the block needs
        // both (C <= 9 gives cg.threads < 16 spb_f; the K1 of the scenes beyond would not run)
        const int threads_f = step_waves == 1 ? 256 : step_waves == 2 ? 512
                                                      : std::max(cg.threads, ((16 * spb_f + 63) / 64) * 64);
        // the step kernel's own start/end timestamps go into K2's events (the launch's dispatch
        // records them): no marker packets in the stream, which cost a few us each in a ~0.1 ms step
        hipEvent_t e1 = tk2 ? ev(1) : nullptr, e2 = tk2 ? ev(2) : nullptr;
        if (fio) {
            if (tk2) (void)hipEventRecord(ev(1), st);
            hipLaunchKernelGGL(k_plan_frame, dim3(1), dim3(threads_f), lds_f, st, *fio, mg, B, P, pv, R, spb_f,
                               rec, adjm, step_waves == 1 ? 1 : 0);
            if (tk2) (void)hipEventRecord(ev(2), st);
        } else if (step_waves == 2) {
            hipExtLaunchKernelGGL(k_step_small512, dim3((unsigned)groups_f), dim3(threads_f), (uint32_t)lds_f, st,
                                  e1, e2, 0u, mg, B, P, pv, R, spb_f, rec, adjm);
        } else {
            hipExtLaunchKernelGGL(k_step_small, dim3((unsigned)groups_f), dim3(threads_f), (uint32_t)lds_f, st,
                                  e1, e2, 0u, mg, B, P, pv, R, spb_f, rec, adjm, step_waves == 1 ? 1 : 0);
        }
        if (tall) (void)hipEventRecord(ev(3), st);
        if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
        return PP_OK;
    }
    if (hipMemsetAsync(gb.count, 0, kPartMax * sizeof(uint32_t), st) != hipSuccess) return PP_ERR_HIP;
    const bool split = ref_direct && !P.emit_paths && !fused && cg.bps == 1 && Dn == 1 &&
                       prep_group(Sv) == 1 && split_on(S);
    g_dbg[PP_DBG_LAST_PARTS].store(1, std::memory_order_relaxed);
    if (split) {
        // NT = streams x chunks parts at group boundaries: part t takes groups [G t / NT, G (t + 1) /
        // NT) and their scenes, on stream t % NS (stream 0: the caller's, else st2[.]); each part its
        // own flagged-group list (count word t, its list from its first group's index on).
        // Chunks run one after another (fork and join per chunk).
        // Timing: each part's kernels by events on its own stream; pp_timing_read counts each stage
        // once per call, as the span from a chunk's first part's start to its last part's end (the
        // parts overlap, so one part's duration understates the stage's throughput), summed over
        // the chunks.
        const int NS = split_parts(S), NC = split_chunks(S), NT = NS * NC;
        if (!W.fork && hipEventCreateWithFlags(&W.fork, hipEventDisableTiming) != hipSuccess) return PP_ERR_HIP;
        for (int k = 0; k < NS - 1; k++)
            if (!W.st2[k] && (hipStreamCreateWithFlags(&W.st2[k], hipStreamNonBlocking) != hipSuccess ||
                              hipEventCreateWithFlags(&W.join[k], hipEventDisableTiming) != hipSuccess))
                return PP_ERR_HIP;
        const int64_t G = cg.groups;
        const bool lmap = mg.n <= kLdsMapMax;
        const size_t lds = lmap ? sizeof(double) * kMapArrays * (size_t)mg.n : 0;
        const size_t lds_a = lmap && mg.atab_lds ? prep_lds_atab(mg.n) : lds;    // k_prep<true, false>
        MapG mga = mg;
        if (!mg.atab_lds) mga.atab = nullptr;
        int launched = 0;     // parts launched (an empty part is skipped; never at >= 2,048 scenes)
        for (int c = 0; c < NC; c++) {
            // fork: the chunk's other streams start behind everything before it on the caller's stream
            if (hipEventRecord(W.fork, st) != hipSuccess) return PP_ERR_HIP;
            for (int k = 0; k < NS - 1; k++)
                if (hipStreamWaitEvent(W.st2[k], W.fork, 0) != hipSuccess) return PP_ERR_HIP;
            for (int h = 0; h < NS; h++) {
                const int t = c * NS + h;
                hipStream_t sh = h == 0 ? st : W.st2[h - 1];
                const int64_t g0 = G * t / NT, g1 = G * (t + 1) / NT;
                const int64_t v0 = std::min<int64_t>(S, g0 * cg.spb), v1 = std::min<int64_t>(S, g1 * cg.spb);
                if (v1 <= v0) continue;
                GroupBits gbh = gb;
                gbh.count = gb.count + t;
                gbh.list = gb.list + g0;
                const int eh = 4 * launched++;
                if (tall) (void)hipEventRecord(ev(eh), sh);
                const unsigned pb = (unsigned)((v1 - v0 + 255) / 256);
                if (srt.rows)         // (the split takes batches without draws: scene = evaluation)
                    hipLaunchKernelGGL(k_sort_cars, dim3(pb), dim3(256), 0, sh, B, srt, v0, v1);
                if (srt.rows) {
                    if (prep_w4(v1 - v0, device)) {
                        if (lmap) hipLaunchKernelGGL((k_prep<true, true, true>), dim3(pb), dim3(256), lds, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                        else hipLaunchKernelGGL((k_prep<false, true, true>), dim3(pb), dim3(256), 0, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                    } else {
                        if (lmap) hipLaunchKernelGGL((k_prep<true, false, true>), dim3(pb), dim3(256), lds_a, sh, mga, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                        else hipLaunchKernelGGL((k_prep<false, false, true>), dim3(pb), dim3(256), 0, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                    }
                } else if (prep_w4(v1 - v0, device)) {
                    if (lmap) hipLaunchKernelGGL((k_prep<true, true>), dim3(pb), dim3(256), lds, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                    else hipLaunchKernelGGL((k_prep<false, true>), dim3(pb), dim3(256), 0, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                } else {
                    if (lmap) hipLaunchKernelGGL((k_prep<true, false>), dim3(pb), dim3(256), lds_a, sh, mga, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                    else hipLaunchKernelGGL((k_prep<false, false>), dim3(pb), dim3(256), 0, sh, mg, B, P, pv, R.info, R.status, gbh, v0, v1, srt);
                }
                if (tk2) (void)hipEventRecord(ev(eh + 1), sh);
                const unsigned nsl = (unsigned)std::min<int64_t>(g1 - g0, 2048);
                hipLaunchKernelGGL((k_cand<false, 1>), dim3((unsigned)(g1 - g0)), dim3(cg.threads), cg.lds, sh, mg, B, P, pv, R,
                                   cg.spb, cg.bps, rec, adjm, W.gbits, G, gbh.list, gbh.count, g0, (double*)nullptr);
                hipLaunchKernelGGL((k_cand<true, 1>), dim3(nsl), dim3(cg.threads), cg.lds, sh, mg, B, P, pv, R,
                                   cg.spb, cg.bps, rec, adjm, W.gbits, G, gbh.list, gbh.count, g0, (double*)nullptr);
                if (tk2) (void)hipEventRecord(ev(eh + 2), sh);
                hipLaunchKernelGGL(k_emit<kEmitRows>, dim3((unsigned)((v1 - v0 + 255) / 256)), dim3(256), 0, sh, B, P, pv, R,
                                   rec, adjm, v0, v1);
                if (tall) (void)hipEventRecord(ev(eh + 3), sh);
            }
            // join: the caller's stream waits for the chunk's other streams
            for (int k = 0; k < NS - 1; k++)
                if (hipEventRecord(W.join[k], W.st2[k]) != hipSuccess || hipStreamWaitEvent(st, W.join[k], 0) != hipSuccess)
                    return PP_ERR_HIP;
        }
        // (the timing record: parts launched, and parts per chunk for the per-chunk spans)
        if (timing) DS.ev_kind.back() |= (launched << 8) | (NC > 1 ? NS << 16 : 0);
        g_dbg[PP_DBG_LAST_PARTS].store(launched, std::memory_order_relaxed);
        if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
        return PP_OK;
    }
    // K1: one lane per evaluation, or a group of G lanes per evaluation for small batches
    {
        const int threads = 256;
        const int G = prep_group(Sv);
        const int64_t blocks = (Sv * G + threads - 1) / threads;
        if (tall) (void)hipEventRecord(ev(0), st);
        const bool lmap = mg.n <= kLdsMapMax;
        const size_t lds = lmap ? sizeof(double) * kMapArrays * (size_t)mg.n : 0;
        const size_t lds_a = lmap && mg.atab_lds ? prep_lds_atab(mg.n) : lds;    // k_prep<true, false>
        MapG mga = mg;
        if (!mg.atab_lds) mga.atab = nullptr;
#define PP_LAUNCH_PREP(KER) \
        if (lmap) hipLaunchKernelGGL(KER<true>, dim3((unsigned)blocks), dim3(threads), lds, st, mg, B, P, pv, R.info, R.status, gb); \
        else hipLaunchKernelGGL(KER<false>, dim3((unsigned)blocks), dim3(threads), 0, st, mg, B, P, pv, R.info, R.status, gb)
        switch (G) {
            case 2: { PP_LAUNCH_PREP(k_prep_g2); break; }
            case 4: { PP_LAUNCH_PREP(k_prep_g4); break; }
            case 8: { PP_LAUNCH_PREP(k_prep_g8); break; }
            case 16: { PP_LAUNCH_PREP(k_prep_g16); break; }
            default: {
                if (srt.rows)
                    hipLaunchKernelGGL(k_sort_cars, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, B, srt, (int64_t)0, S);
                if (srt.rows) {
                    if (prep_w4(Sv, device)) {
                        if (lmap) hipLaunchKernelGGL((k_prep<true, true, true>), dim3((unsigned)blocks), dim3(threads), lds, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                        else hipLaunchKernelGGL((k_prep<false, true, true>), dim3((unsigned)blocks), dim3(threads), 0, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                    } else {
                        if (lmap) hipLaunchKernelGGL((k_prep<true, false, true>), dim3((unsigned)blocks), dim3(threads), lds_a, st, mga, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                        else hipLaunchKernelGGL((k_prep<false, false, true>), dim3((unsigned)blocks), dim3(threads), 0, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                    }
                } else if (prep_w4(Sv, device)) {
                    if (lmap) hipLaunchKernelGGL((k_prep<true, true>), dim3((unsigned)blocks), dim3(threads), lds, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                    else hipLaunchKernelGGL((k_prep<false, true>), dim3((unsigned)blocks), dim3(threads), 0, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                } else {
                    if (lmap) hipLaunchKernelGGL((k_prep<true, false>), dim3((unsigned)blocks), dim3(threads), lds_a, st, mga, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                    else hipLaunchKernelGGL((k_prep<false, false>), dim3((unsigned)blocks), dim3(threads), 0, st, mg, B, P, pv, R.info, R.status, gb, (int64_t)0, Sv, srt);
                }
                break;
            }
        }
#undef PP_LAUNCH_PREP
    }
    // K2 (+ K4 for small batches in reference mode: k_cand_small)
    {
        const unsigned nb = (unsigned)cg.groups;
        const unsigned nslow = (unsigned)std::min<int64_t>(cg.groups, 2048);
        const int64_t ng = cg.groups;
        if (tk2) (void)hipEventRecord(ev(1), st);
#define PP_LAUNCH_CAND(MODE)                                                                              \
        hipLaunchKernelGGL((k_cand<false, MODE>), dim3(nb), dim3(cg.threads), cand_lds, st, mg, B, P, pv, R, \
                           cg.spb, cg.bps, rec, adjm, W.gbits, ng, gb.list, gb.count, (int64_t)0, wslot);   \
        hipLaunchKernelGGL((k_cand<true, MODE>), dim3(nslow), dim3(cg.threads), cand_lds, st, mg, B, P, pv, R, \
                           cg.spb, cg.bps, rec, adjm, W.gbits, ng, gb.list, gb.count, (int64_t)0, wslot)
        if (P.emit_paths) { PP_LAUNCH_CAND(2); }
        else if (ref_direct && fused) {
            hipLaunchKernelGGL(k_cand_small, dim3(nb), dim3(cg.threads), cg.lds, st, mg, B, P, pv, R,
                               cg.spb, rec, adjm, W.gbits);
        }
        else if (ref_direct) { PP_LAUNCH_CAND(1); }
        else { PP_LAUNCH_CAND(0); }
#undef PP_LAUNCH_CAND
    }
    if (tk2) (void)hipEventRecord(ev(2), st);
    // K4 (reference mode, winner-only output): replay the winners' recorded paths
    if (ref_direct && !P.emit_paths && !emit_in) {
        if (S <= kEmitSmall) {     // latency regime: 64-lane blocks over more CUs, 16 steps per load round
            const int64_t blocks = (S + 63) / 64;
            hipLaunchKernelGGL(k_emit<16>, dim3((unsigned)blocks), dim3(64), 0, st, B, P, pv, R, rec, adjm, (int64_t)0, S);
        } else {
            const int64_t blocks = (S + 255) / 256;
            hipLaunchKernelGGL(k_emit<kEmitRows>, dim3((unsigned)blocks), dim3(256), 0, st, B, P, pv, R, rec, adjm, (int64_t)0, S);
        }
    }
    // K3 (comfort mode, or any mode with draws): argmin + winner path
    if (!ref_direct) {
        const int64_t blocks = (S + kWinBlock - 1) / kWinBlock;
        if (wslot) {
            const unsigned b256 = (unsigned)((S + 255) / 256);
            hipLaunchKernelGGL((k_winner_st<false>), dim3(b256), dim3(256), 0, st, B, P, pv, R, (const double*)wslot);
            hipLaunchKernelGGL((k_winner_st<true>), dim3(b256), dim3(256), 0, st, B, P, pv, R, (const double*)wslot);
        } else {
            hipLaunchKernelGGL((k_winner<false>), dim3((unsigned)blocks), dim3(kWinBlock), 0, st, mg, B, P, pv, R);
            hipLaunchKernelGGL((k_winner<true>), dim3((unsigned)blocks), dim3(kWinBlock), 0, st, mg, B, P, pv, R);
        }
    }
    if (tall) (void)hipEventRecord(ev(3), st);
    if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
    return PP_OK;
}

}  // namespace
extern "C" {

int32_t pp_eval(pp_map* M, const pp_scene_batch* in, const pp_params* prm, pp_result* out,
                int32_t device, void* hip_stream) {
    return eval_impl(M, in, prm, out, device, hip_stream, nullptr);
}

int32_t pp_debug_set(int32_t key, int32_t value) {
    bool ok = false;
    switch (key) {
        case PP_DBG_PREP_GROUP: ok = prep_group_ok(value); break;
        case PP_DBG_PREP_WAVES: ok = value == 0 || value == 3 || value == 4; break;
        case PP_DBG_SHAPE: ok = value >= 0 && value <= PP_SHAPE_STEP; break;
        case PP_DBG_POISON: ok = value == 0 || value == 1; break;
        case PP_DBG_SPLIT: ok = value >= 0 && value <= 2; break;
        case PP_DBG_SORT_CARS: ok = value >= 0 && value <= 2; break;
        default: break;       // (PP_DBG_LAST_PARTS is read-only)
    }
    if (!ok) return PP_ERR_ARG;
    g_dbg[key].store(value, std::memory_order_relaxed);
    return PP_OK;
}

int32_t pp_debug_get(int32_t key) { return key >= 0 && key < PP_DBG_KEYS ? dbg(key) : PP_ERR_ARG; }

int32_t pp_timing_enable(pp_map* M, int32_t device, int32_t enable) {
    if (!M || device < 0 || device >= kMaxDev) return PP_ERR_ARG;
    std::lock_guard<std::mutex> lk(M->mu);
    DevState& D = M->dev[device];
    D.timing = enable == PP_TIMING_K2 ? 2 : (enable != 0 ? 1 : 0);
    if (D.timing) {
        // events made now, outside any timed region: 2,048 calls of K2-only timing (2 events each,
        // 2 per part when split) or 1,024 of all-kernel timing (4 per part); pp_eval takes the
        // events it records from this pool, pp_timing_read returns them
        DeviceGuard g(device);
        const int rc = dev_init(M, device);       // (pp_map_destroy frees the events of initialised devices)
        if (rc) return rc;
        while (D.ev_pool.size() + D.ev_rec.size() < 4 * kSplitMax * 256) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return PP_ERR_HIP;
            D.ev_pool.push_back(e);
        }
    }
    return PP_OK;
}

int32_t pp_timing_read(pp_map* M, int32_t device, double* ms3, int64_t* launches3) {
    if (!M || device < 0 || device >= kMaxDev || !ms3 || !launches3) return PP_ERR_ARG;
    std::lock_guard<std::mutex> lk(M->mu);
    DevState& D = M->dev[device];
    DeviceGuard g(device);
    for (int k = 0; k < 3; k++) { ms3[k] = 0; launches3[k] = 0; }
    int rc = PP_OK;
    constexpr int EG = 4 * kPartMax;
    const size_t ng = D.ev_rec.size() / EG;
    // signed milliseconds from a to b (either order)
    auto dt = [&](hipEvent_t a, hipEvent_t b, float& t) {
        if (!a || !b) { rc = PP_ERR_HIP; return false; }
        if (hipEventElapsedTime(&t, a, b) == hipSuccess) return true;
        if (hipEventElapsedTime(&t, b, a) == hipSuccess) { t = -t; return true; }
        rc = PP_ERR_HIP;
        return false;
    };
    for (size_t i = 0; i < ng; i++) {
        const int kind = D.ev_kind[i], parts = (kind >> 8) & 0xFF, np = parts ? parts : 1;
        const int per = (kind >> 16) & 0xF, pc = per ? per : np;    // parts per chunk
        const bool k2only = (kind & 16) != 0;
        hipEvent_t* e0 = &D.ev_rec[EG * i];
        for (int h = 0; h < np; h++) {
            hipEvent_t last = k2only ? e0[4 * h + 2] : e0[4 * h + 3];
            if (!last || hipEventSynchronize(last) != hipSuccess) rc = PP_ERR_HIP;
        }
        // stage k (0: K1, 1: K2, 2: K3/K4) of a call: per chunk, from its earliest start to its
        // latest end over the chunk's parts (one stream: the kernel's own interval; a split call's
        // parts overlap, and the stage's time is the span they cover together, as in a kernel
        // trace), summed over the chunks; one launch per call
        for (int k = 0; k < 3; k++) {
            if (k != 1 && (k2only || (k == 0 && (kind & 32)) || (k == 2 && !(kind & 1)))) continue;
            float sum = 0;
            bool ok = true;
            for (int c0 = 0; c0 < np && ok; c0 += pc) {
                float lo = 0, hi = 0;
                for (int h = c0; h < std::min(np, c0 + pc) && ok; h++) {
                    float a, b;
                    ok = dt(e0[1], e0[4 * h + k], a) && dt(e0[1], e0[4 * h + k + 1], b);
                    if (ok) { lo = h == c0 ? a : std::min(lo, a); hi = h == c0 ? b : std::max(hi, b); }
                }
                sum += hi - lo;
            }
            if (ok) { ms3[k] += sum; launches3[k]++; }
        }
        for (int k = 0; k < EG; k++)
            if (D.ev_rec[EG * i + k]) D.ev_pool.push_back(D.ev_rec[EG * i + k]);
    }
    D.ev_rec.clear();
    D.ev_kind.clear();
    return rc;
}

int32_t pp_synth_scenes(pp_map* M, uint64_t seed, int64_t first_scene, pp_scene_batch* out,
                        int32_t device, void* hip_stream) {
    if (!M || !out || device < 0 || device >= kMaxDev || out->n_scenes < 0 || first_scene < 0) return PP_ERR_ARG;
    if (out->car_stride < ppsynth::kSynthCars) return PP_ERR_ARG;
    if (out->n_scenes == 0) return PP_OK;
    DeviceGuard g(device);
    ppsynth::LaneTables T;
    {
        std::lock_guard<std::mutex> lk(M->mu);
        const int rc = dev_init(M, device);
        if (rc) return rc;
        T = lane_tables(M->dev[device].lanetab, M->n);
    }
    const ppsynth::OutBatch o = out_batch(out);
    const int threads = 256;
    const int64_t blocks = (o.S + threads - 1) / threads;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)hip_stream, T, seed, first_scene, o);
    if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
    return PP_OK;
}

int32_t pp_synth_scenes_host(const pp_map* M, uint64_t seed, int64_t first_scene, pp_scene_batch* out) {
    if (!M || !out || out->n_scenes < 0 || first_scene < 0 || out->car_stride < ppsynth::kSynthCars) return PP_ERR_ARG;
    const ppsynth::LaneTables T = lane_tables(M->lanetab.data(), M->n);
    const ppsynth::OutBatch o = out_batch(out);
    for (int64_t s = 0; s < o.S; s++) ppsynth::synth_scene(T, seed, first_scene + s, s, o);
    return PP_OK;
}

int32_t pp_synth_traffic(pp_map* M, uint64_t seed, int64_t first_scene, pp_scene_batch* tel,
                         pp_traffic* out, int32_t device, void* hip_stream) {
    if (!M || !tel || device < 0 || device >= kMaxDev || tel->n_scenes < 0 || first_scene < 0 ||
        tel->car_stride < ppsynth::kSynthCars || !traffic_ok(out, tel) ||
        (tel->tab_valid && (tel->tab_slots < ppsynth::kSynthCars || tel->tab_slots > PP_MAX_CARS)))
        return PP_ERR_ARG;
    if (tel->n_scenes == 0) return PP_OK;
    DeviceGuard g(device);
    ppsynth::LaneTables T;
    {
        std::lock_guard<std::mutex> lk(M->mu);
        const int rc = dev_init(M, device);
        if (rc) return rc;
        T = lane_tables(M->dev[device].lanetab, M->n);
    }
    out->n_cars = ppsynth::kSynthCars;
    const ppsynth::OutBatch o = out_batch(tel);
    const int64_t blocks = (o.S + 255) / 256;
    hipLaunchKernelGGL(k_synth_traffic, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hip_stream, T,
                       seed, first_scene, o, traffic_view(out, o.S), *tel);
    if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
    return PP_OK;
}

int32_t pp_synth_traffic_host(const pp_map* M, uint64_t seed, int64_t first_scene, pp_scene_batch* tel,
                              pp_traffic* out) {
    if (!M || !tel || tel->n_scenes < 0 || first_scene < 0 || tel->car_stride < ppsynth::kSynthCars ||
        !traffic_ok(out, tel) ||
        (tel->tab_valid && (tel->tab_slots < ppsynth::kSynthCars || tel->tab_slots > PP_MAX_CARS)))
        return PP_ERR_ARG;
    const ppsynth::LaneTables T = lane_tables(M->lanetab.data(), M->n);
    out->n_cars = ppsynth::kSynthCars;
    const ppsynth::OutBatch o = out_batch(tel);
    const ppsynth::TrafficV tv = traffic_view(out, o.S);
    for (int64_t s = 0; s < o.S; s++) {
        ppsynth::synth_scene(T, seed, first_scene + s, s, o, &tv);
        for (int j = 0; tel->tab_valid && j < tel->tab_slots; j++) {
            tel->tab_valid[(int64_t)j * o.S + s] = 0;
            if (tel->tab_id) tel->tab_id[(int64_t)j * o.S + s] = j;
        }
    }
    return PP_OK;
}

int32_t pp_rollout(pp_map* M, pp_scene_batch* tel, pp_traffic* traffic, const pp_params* prm,
                   const pp_rollout_cfg* cfg, pp_result* res, pp_rollout_log* log, int32_t device,
                   void* hip_stream) {
    if (!M || !tel || !prm || !cfg || !res || device < 0 || device >= kMaxDev || !traffic_ok(traffic, tel))
        return PP_ERR_ARG;
    if (cfg->n_frames < 0 || cfg->consume < 1 || !(cfg->sensor_range >= 0) || prm->n_draws > 1 ||
        prm->emit_paths || !tel->tab_valid || !tel->tab_lane || !tel->tab_s || !tel->tab_d ||
        !tel->tab_vs || !tel->tab_vd || !tel->tab_vx || !tel->tab_vy || tel->car_stride < traffic->n_cars ||
        tel->tab_slots < traffic->n_cars)
        return PP_ERR_ARG;
    if (log && log->plan_x && !log->plan_y) return PP_ERR_ARG;
    if (tel->n_scenes == 0 || cfg->n_frames == 0) return PP_OK;
    DeviceGuard g(device);
    ppsynth::LaneTables T;
    {
        std::lock_guard<std::mutex> lk(M->mu);
        const int rc = dev_init(M, device);
        if (rc) return rc;
        T = lane_tables(M->dev[device].lanetab, M->n);
    }
    SimArgs A;
    A.consume = cfg->consume;
    A.range2 = cfg->sensor_range * cfg->sensor_range;
    if (log) A.log = *log; else memset(&A.log, 0, sizeof(A.log));
    const ppsynth::TrafficV tv = traffic_view(traffic, tel->n_scenes);
    const int64_t blocks = (tel->n_scenes + 255) / 256;
    for (int f = 0; f < cfg->n_frames; f++) {
        const int rc = pp_eval(M, tel, prm, res, device, hip_stream);
        if (rc != PP_OK) return rc;
        A.frame = f;
        hipLaunchKernelGGL(k_sim, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)hip_stream, T, *tel,
                           tv, *prm, *res, A);
        if (hipGetLastError() != hipSuccess) return PP_ERR_HIP;
    }
    return PP_OK;
}

// Host-memory batch (the batched onMessage): stage the scenes (and their car table) into device
// memory, pp_eval, copy results (and the updated table) back. Synchronous.
// pp_plan_batch_host stages batches up to this many scenes through its pinned mirror
constexpr int64_t kStageMirrorMax = 512;
int32_t pp_plan_batch_host(pp_map* M, int32_t device, pp_scene_batch* hin, const pp_params* prm,
                           pp_result* hout, void* hip_stream) {
    if (!M || !hin || !prm || !hout || device < 0 || device >= kMaxDev || !params_ok(prm) || prm->emit_paths ||
        hin->n_scenes < 0 || hin->car_stride < 0 || hin->car_stride > PP_MAX_CARS)
        return PP_ERR_ARG;
    if (!hout->winner || !hout->n_out || !hout->next_x || !hout->next_y || !hout->cost || !hout->status)
        return PP_ERR_ARG;
    const int64_t S = hin->n_scenes;
    if (S == 0) return PP_OK;
    const int J = hin->car_stride, N = prm->n_points;
    const int C = n_draws(prm) * NL * prm->n_speeds;
    const bool tab = hin->tab_valid != nullptr;
    // staging layout: doubles first, then 4-byte fields
    const int TS = tab ? hin->tab_slots : 0;
    if (tab && (TS < 0 || TS > PP_MAX_CARS)) return PP_ERR_ARG;
    // every host pointer the staging copies touch (small batches memcpy them on the host, so a
    // NULL here must be refused before staging, not left to the copy)
    if (!hin->ego_x || !hin->ego_y || !hin->ego_yaw_deg || !hin->ego_speed_mph || !hin->prev_x || !hin->prev_y ||
        !hin->n_prev || !hin->prev_target_lane || !hin->n_cars)
        return PP_ERR_ARG;
    if (J > 0 && (!hin->car_id || !hin->car_x || !hin->car_y || !hin->car_vx || !hin->car_vy)) return PP_ERR_ARG;
    if (tab && TS > 0 && (!hin->tab_lane || !hin->tab_s || !hin->tab_d || !hin->tab_vs || !hin->tab_vd ||
                          !hin->tab_vx || !hin->tab_vy))
        return PP_ERR_ARG;
    const size_t nd = (size_t)S * (4 + 2 * PP_PREV_KEEP + 4 * J + 6 * TS + 2 * N + C);
    const size_t ni = (size_t)S * (3 + J + 3 * TS + 3);
    const size_t bytes = nd * 8 + ni * 4 + 256;
    DeviceGuard g(device);
    hipStream_t st = (hipStream_t)hip_stream;
    std::lock_guard<std::mutex> stage_lock(M->dev[device].stage_mu);
    char* base;
    char* mirror;                 // pinned host mirror of the staging buffer (same offsets)
    {
        std::lock_guard<std::mutex> lk(M->mu);
        int rc = dev_init(M, device);
        if (rc) return rc;
        DevState& D = M->dev[device];
        if (D.stage_cap < bytes) {
            if (D.stage) { (void)hipDeviceSynchronize(); (void)hipFree(D.stage); D.stage = nullptr; D.stage_cap = 0; }
            if (D.stage_host) { (void)hipHostFree(D.stage_host); D.stage_host = nullptr; }
            if (hipMalloc(&D.stage, bytes) != hipSuccess) return PP_ERR_NOMEM;
            if (hipHostMalloc(&D.stage_host, bytes, hipHostMallocDefault) != hipSuccess) {
                (void)hipFree(D.stage); D.stage = nullptr; return PP_ERR_NOMEM;
            }
            D.stage_cap = bytes;
        }
        base = (char*)D.stage;
        mirror = (char*)D.stage_host;
    }
    double* dp = (double*)base;
    int32_t* ip = (int32_t*)(base + nd * 8);
    auto takeD = [&](size_t n) { double* r = dp; dp += n; return r; };
    auto takeI = [&](size_t n) { int32_t* r = ip; ip += n; return r; };
    bool ok = true;
    // Small batches (latency): inputs are gathered into the pinned mirror; the input fields lead
    // each region (doubles, then ints), so one copy per region moves them, and one per region
    // brings the outputs back. Large batches (bandwidth): one asynchronous copy per field straight
    // from and to the caller's buffers (the extra host memcpy through the mirror costs more there).
    const bool small = S <= kStageMirrorMax;
    auto h2d = [&](void* d, const void* h, size_t n) {
        if (!n) return;
        if (small) memcpy(mirror + ((char*)d - base), h, n);
        else if (hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st) != hipSuccess) ok = false;
    };
    pp_scene_batch B;
    memset(&B, 0, sizeof(B));
    B.n_scenes = S; B.car_stride = J;
    double* ego = takeD(4 * S);
    B.ego_x = ego; B.ego_y = ego + S; B.ego_yaw_deg = ego + 2 * S; B.ego_speed_mph = ego + 3 * S;
    h2d(ego, hin->ego_x, 8 * S); h2d(ego + S, hin->ego_y, 8 * S);
    h2d(ego + 2 * S, hin->ego_yaw_deg, 8 * S); h2d(ego + 3 * S, hin->ego_speed_mph, 8 * S);
    double* pxy = takeD(2 * PP_PREV_KEEP * S);
    B.prev_x = pxy; B.prev_y = pxy + PP_PREV_KEEP * S;
    h2d(pxy, hin->prev_x, 8 * PP_PREV_KEEP * S); h2d(pxy + PP_PREV_KEEP * S, hin->prev_y, 8 * PP_PREV_KEEP * S);
    double* cars = takeD(4 * (size_t)J * S);
    B.car_x = cars; B.car_y = cars + J * S; B.car_vx = cars + 2 * J * S; B.car_vy = cars + 3 * J * S;
    if (J) {
        h2d(cars, hin->car_x, 8 * J * S); h2d(cars + J * S, hin->car_y, 8 * J * S);
        h2d(cars + 2 * J * S, hin->car_vx, 8 * J * S); h2d(cars + 3 * J * S, hin->car_vy, 8 * J * S);
    }
    double* tabd = nullptr;
    if (tab) {
        tabd = takeD(6 * (size_t)TS * S);
        const double* src[6] = {hin->tab_s, hin->tab_d, hin->tab_vs, hin->tab_vd, hin->tab_vx, hin->tab_vy};
        double** dst[6] = {&B.tab_s, &B.tab_d, &B.tab_vs, &B.tab_vd, &B.tab_vx, &B.tab_vy};
        for (int k = 0; k < 6; k++) { *dst[k] = tabd + k * (size_t)TS * S; h2d(*dst[k], src[k], 8 * (size_t)TS * S); }
        B.tab_slots = TS;
    }
    double* nxy = takeD(2 * (size_t)N * S);
    double* cost = takeD((size_t)C * S);
    int32_t* ints = takeI(3 * S);
    B.n_prev = ints; B.prev_target_lane = ints + S; B.n_cars = ints + 2 * S;
    h2d(ints, hin->n_prev, 4 * S); h2d(ints + S, hin->prev_target_lane, 4 * S); h2d(ints + 2 * S, hin->n_cars, 4 * S);
    int32_t* cid = takeI((size_t)J * S);
    B.car_id = cid;
    h2d(cid, hin->car_id, 4 * J * S);
    int32_t* tabi = nullptr;
    if (tab) {
        tabi = takeI(3 * (size_t)TS * S);
        B.tab_valid = tabi; B.tab_lane = tabi + (size_t)TS * S;
        h2d(tabi, hin->tab_valid, 4 * (size_t)TS * S); h2d(tabi + (size_t)TS * S, hin->tab_lane, 4 * (size_t)TS * S);
        if (hin->tab_id) { B.tab_id = tabi + 2 * (size_t)TS * S; h2d(B.tab_id, hin->tab_id, 4 * (size_t)TS * S); }
    }
    int32_t* outi = takeI(3 * S);
    pp_result R;
    memset(&R, 0, sizeof(R));
    R.winner = outi; R.n_out = outi + S; R.status = (uint32_t*)(outi + 2 * S);
    R.next_x = nxy; R.next_y = nxy + (size_t)N * S; R.cost = cost;
    const char* d_in_end = (const char*)nxy;           // doubles: inputs [base, nxy)
    const char* i_beg = base + nd * 8;                  // ints: inputs [i_beg, outi)
    const char* d_out_beg = tab ? (const char*)tabd : (const char*)nxy;   // outputs: (tables,) plans, costs
    const char* d_out_end = (const char*)(cost + (size_t)C * S);
    const char* i_out_beg = tab ? (const char*)tabi : (const char*)outi;
    const char* i_out_end = (const char*)(outi + 3 * S);
    auto copy = [&](const char* lo, const char* hi, bool in) {
        if (hi <= lo) return;
        char* h = mirror + (lo - base);
        if (hipMemcpyAsync(in ? (void*)lo : (void*)h, in ? (const void*)h : (const void*)lo, (size_t)(hi - lo),
                           in ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, st) != hipSuccess) ok = false;
    };
    if (small) { copy(base, d_in_end, true); copy(i_beg, (const char*)outi, true); }
    if (!ok) return PP_ERR_HIP;
    int rc = pp_eval(M, &B, prm, &R, device, hip_stream);
    if (rc != PP_OK) return rc;
    if (small && dbg(PP_DBG_POISON)) {   // the mirror's pure-output regions (inputs may still be in flight)
        memset(mirror + ((const char*)nxy - base), 0xFF, (size_t)(d_out_end - (const char*)nxy));
        memset(mirror + ((const char*)outi - base), 0xFF, (size_t)(i_out_end - (const char*)outi));
    }
    if (small) {
        copy(d_out_beg, d_out_end, false);
        copy(i_out_beg, i_out_end, false);
        if (!ok || hipStreamSynchronize(st) != hipSuccess) return PP_ERR_HIP;
    }
    auto d2h = [&](void* h, const void* d, size_t n) {
        if (!n) return;
        if (small) memcpy(h, mirror + ((const char*)d - base), n);
        else if (hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st) != hipSuccess) ok = false;
    };
    d2h(hout->winner, R.winner, 4 * S); d2h(hout->n_out, R.n_out, 4 * S); d2h(hout->status, R.status, 4 * S);
    d2h(hout->next_x, R.next_x, 8 * (size_t)N * S); d2h(hout->next_y, R.next_y, 8 * (size_t)N * S);
    d2h(hout->cost, R.cost, 8 * (size_t)C * S);
    if (tab) {
        double* dstd[6] = {hin->tab_s, hin->tab_d, hin->tab_vs, hin->tab_vd, hin->tab_vx, hin->tab_vy};
        for (int k = 0; k < 6; k++) d2h(dstd[k], tabd + k * (size_t)TS * S, 8 * (size_t)TS * S);
        d2h(hin->tab_valid, tabi, 4 * (size_t)TS * S); d2h(hin->tab_lane, tabi + (size_t)TS * S, 4 * (size_t)TS * S);
    }
    if (!small && (!ok || hipStreamSynchronize(st) != hipSuccess)) return PP_ERR_HIP;
    return PP_OK;
}

int32_t pp_plan_reset(pp_map* M, int32_t device) {
    if (!M || device < 0 || device >= kMaxDev) return PP_ERR_ARG;
    std::lock_guard<std::mutex> lk(M->dev[device].frame_mu);
    M->dev[device].plan_table.cars.clear();
    return PP_OK;
}

// One telemetry frame (the onMessage replacement): C = 3 (one speed: max_speed), reference mode.
#ifdef PP_FRAME_PROF
// diagnostic builds (-DPP_FRAME_PROF): per-frame host and device intervals, summed (us) — host:
// staging until the launch, the launch call, launch-to-done, done-to-return; device (100 MHz
// clock): input copy, the frame's body, output copy; and the frame count. pp_frame_prof_read
// returns and clears them.
static double g_fprof[8];
static double fprof_now() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int32_t pp_frame_prof_read(double* out8) {
    for (int i = 0; i < 8; i++) { out8[i] = g_fprof[i]; g_fprof[i] = 0; }
    return PP_OK;
}
#endif
int32_t pp_plan_frame(pp_map* M, int32_t device, double ego_x, double ego_y, double ego_yaw_deg,
                      double ego_speed_mph, const double* prev_x, const double* prev_y, int32_t n_prev,
                      const int32_t* car_id, const double* car_x, const double* car_y,
                      const double* car_vx, const double* car_vy, int32_t n_cars,
                      int32_t* target_lane, double* next_x, double* next_y, int32_t* n_out) {
    if (!M || !target_lane || !next_x || !next_y || !n_out || n_cars < 0 || n_cars > PP_MAX_CARS ||
        device < 0 || device >= kMaxDev || (n_prev > 0 && (!prev_x || !prev_y)) ||
        (n_cars > 0 && (!car_id || !car_x || !car_y || !car_vx || !car_vy)))
        return PP_ERR_ARG;
    if (*target_lane < 0 || *target_lane >= NL) return PP_ERR_ARG;
#ifdef PP_FRAME_PROF
    const double h0 = fprof_now();
#endif
    // host staging: one scene, SoA with S = 1 (std::map order: stable sort by id, last row of a
    // duplicated id wins as in `sensor_fusion_cars[id]` assignment, src/main.cpp:1329)
    struct Row { int32_t id; double x, y, vx, vy; };
    std::vector<Row> rows;
    for (int j = 0; j < n_cars; j++) {
        bool dup = false;
        for (auto& r : rows) if (r.id == car_id[j]) { r = {car_id[j], car_x[j], car_y[j], car_vx[j], car_vy[j]}; dup = true; }
        if (!dup) rows.push_back({car_id[j], car_x[j], car_y[j], car_vx[j], car_vy[j]});
    }
    std::stable_sort(rows.begin(), rows.end(), [](const Row& a, const Row& b) { return a.id < b.id; });
    const int nc = (int)rows.size();
    // device scratch layout (bytes): doubles then ints, then the scene info (the target lane)
    constexpr int N = 50;
    constexpr int TS = PP_MAX_CARS;
    struct Frame {
        double ego[4], px[PP_PREV_KEEP], py[PP_PREV_KEEP], cx[PP_MAX_CARS], cy[PP_MAX_CARS],
            cvx[PP_MAX_CARS], cvy[PP_MAX_CARS];
        double nx[N], ny[N], cost[NL];
        double ts[TS], td[TS], tvs[TS], tvd[TS], tvx[TS], tvy[TS];        // the car table's slots
        int32_t tid[TS], tvalid[TS], tlane[TS];
        int32_t nprev, ptl, ncars, cid[PP_MAX_CARS], winner, nout;
        uint32_t status;
        pp_scene_info info;
    };
    DeviceGuard g(device);
    std::lock_guard<std::mutex> frame_lock(M->dev[device].frame_mu);
    DevState& DS = M->dev[device];
    Frame* d = nullptr;
    constexpr size_t kFlagOff = (sizeof(Frame) + 63) / 64 * 64;
    {   // per-device scratch, made once: the device frame, its pinned host copy, the frame stream
        std::lock_guard<std::mutex> lk(M->mu);
        int rc = dev_init(M, device);
        if (rc) return rc;
        // (both copies kFlagOff bytes: the 16-B units of the last fields may pass sizeof(Frame))
        if (!DS.frame && hipMalloc(&DS.frame, kFlagOff) != hipSuccess) return PP_ERR_NOMEM;
        if (!DS.frame_host) {
            if (hipHostMalloc(&DS.frame_host, kFlagOff + 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
                return PP_ERR_NOMEM;
            memset(DS.frame_host, 0, kFlagOff + 64);
            DS.frame_seq = 0;
        }
        if (!DS.frame_stream && hipStreamCreateWithFlags(&DS.frame_stream, hipStreamNonBlocking) != hipSuccess)
            return PP_ERR_HIP;
        d = (Frame*)DS.frame;
    }
    Frame& h = *(Frame*)DS.frame_host;
    volatile uint32_t* flag = (volatile uint32_t*)((char*)DS.frame_host + kFlagOff);
    // (only the words the frame's ranges carry are written: the previous path's unused tail is
    // zeroed, every other input range is filled below)
    memset(h.px, 0, sizeof h.px); memset(h.py, 0, sizeof h.py);
    const bool poison = dbg(PP_DBG_POISON) != 0;
    if (poison) {     // the outputs' staging starts NaN-filled (pp_eval poisons them on the device too)
        memset(h.nx, 0xFF, sizeof h.nx); memset(h.ny, 0xFF, sizeof h.ny); memset(h.cost, 0xFF, sizeof h.cost);
        memset(&h.winner, 0xFF, sizeof h.winner); memset(&h.nout, 0xFF, sizeof h.nout);
        memset(&h.status, 0xFF, sizeof h.status); memset(&h.info, 0xFF, sizeof h.info);
    }
    h.ego[0] = ego_x; h.ego[1] = ego_y; h.ego[2] = ego_yaw_deg; h.ego[3] = ego_speed_mph;
    for (int i = 0; i < PP_PREV_KEEP && i < n_prev; i++) { h.px[i] = prev_x[i]; h.py[i] = prev_y[i]; }
    h.nprev = n_prev; h.ptl = *target_lane; h.ncars = nc;
    for (int j = 0; j < nc; j++) {
        h.cid[j] = rows[j].id; h.cx[j] = rows[j].x; h.cy[j] = rows[j].y; h.cvx[j] = rows[j].vx; h.cvy[j] = rows[j].vy;
    }
    // the reference's std::map, laid out over the union of its ids and this frame's (any ints)
    const pptab::Slots hs = {1, h.tid, h.tvalid, h.tlane, h.ts, h.td, h.tvs, h.tvd, h.tvx, h.tvy};
    const int nu = DS.plan_table.union_size(h.cid, nc);
    if (nu > TS) return PP_ERR_ARG;                     // more than PP_MAX_CARS distinct cars
    const int nslots = DS.plan_table.layout(h.cid, nc, hs, 0, nu, poison);
    if (nslots < 0) return PP_ERR_ARG;
    hipStream_t st = DS.frame_stream;
    pp_scene_batch B;
    memset(&B, 0, sizeof(B));
    B.n_scenes = 1; B.car_stride = PP_MAX_CARS;
    B.ego_x = &d->ego[0]; B.ego_y = &d->ego[1]; B.ego_yaw_deg = &d->ego[2]; B.ego_speed_mph = &d->ego[3];
    B.prev_x = d->px; B.prev_y = d->py; B.n_prev = &d->nprev; B.prev_target_lane = &d->ptl;
    B.n_cars = &d->ncars; B.car_id = d->cid; B.car_x = d->cx; B.car_y = d->cy; B.car_vx = d->cvx; B.car_vy = d->cvy;
    B.tab_slots = nslots; B.tab_id = d->tid;
    B.tab_valid = d->tvalid; B.tab_lane = d->tlane; B.tab_s = d->ts; B.tab_d = d->td;
    B.tab_vs = d->tvs; B.tab_vd = d->tvd; B.tab_vx = d->tvx; B.tab_vy = d->tvy;
    pp_params P;
    pp_params_default(&P);
    P.n_speeds = 1;
    pp_result R;
    memset(&R, 0, sizeof(R));
    R.winner = &d->winner; R.n_out = &d->nout; R.next_x = d->nx; R.next_y = d->ny; R.cost = d->cost;
    R.status = &d->status; R.info = &d->info;
    // The frame's words that carry data: inputs (ego, previous path, this frame's rows, the table's
    // nslots slots) and outputs (plan, costs, winner / count / status / info, the slots again).
    FrameIO io;
    memset(&io, 0, offsetof(FrameIO, inl));
    // (each field's bytes rounded out to whole 16-B units: the extra words are other fields of the
    // frame — inputs the kernel overwrites nothing of, outputs the host does not read — and a unit
    // range touching the previous one joins it)
    bool fio_full = false;        // a range beyond the kernel argument's kFioMax (never: 15 in, 10 out)
    auto add = [&](bool in, const void* p, size_t bytes) {
        if (!bytes) return;
        const size_t b0 = (size_t)((const char*)p - (const char*)&h);
        const uint32_t u0 = (uint32_t)(b0 / 16), u1 = (uint32_t)((b0 + bytes + 15) / 16);
        int& n = in ? io.n_in : io.n_out;
        uint32_t* off = in ? io.in_off : io.out_off;
        uint32_t* len = in ? io.in_len : io.out_len;
        if (n > 0 && u0 <= off[n - 1] + len[n - 1] && u0 >= off[n - 1]) {
            if (u1 > off[n - 1] + len[n - 1]) len[n - 1] = u1 - off[n - 1];
            return;
        }
        if (n >= kFioMax) { fio_full = true; return; }
        off[n] = u0; len[n] = u1 - u0;
        n++;
    };
    const size_t ns = (size_t)nslots, ncs = (size_t)nc;
    add(true, h.ego, sizeof h.ego + sizeof h.px + sizeof h.py);   // ego, px, py: adjacent
    add(true, h.cx, 8 * ncs); add(true, h.cy, 8 * ncs); add(true, h.cvx, 8 * ncs); add(true, h.cvy, 8 * ncs);
    add(true, h.ts, 8 * ns); add(true, h.td, 8 * ns); add(true, h.tvs, 8 * ns); add(true, h.tvd, 8 * ns);
    add(true, h.tvx, 8 * ns); add(true, h.tvy, 8 * ns);
    add(true, h.tid, 4 * ns); add(true, h.tvalid, 4 * ns); add(true, h.tlane, 4 * ns);
    add(true, &h.nprev, 4 * (3 + ncs));                          // nprev, ptl, ncars, cid[nc]: adjacent
    add(false, h.nx, sizeof h.nx + sizeof h.ny + sizeof h.cost);  // nx, ny, cost: adjacent
    add(false, h.ts, 8 * ns); add(false, h.td, 8 * ns); add(false, h.tvs, 8 * ns); add(false, h.tvd, 8 * ns);
    add(false, h.tvx, 8 * ns); add(false, h.tvy, 8 * ns);
    add(false, h.tvalid, 4 * ns); add(false, h.tlane, 4 * ns);
    add(false, &h.winner, (size_t)((const char*)(&h.info + 1) - (const char*)&h.winner));   // winner .. info
    static_assert(offsetof(Frame, px) == offsetof(Frame, ego) + sizeof(double) * 4 &&
                  offsetof(Frame, py) == offsetof(Frame, px) + sizeof(double) * PP_PREV_KEEP &&
                  offsetof(Frame, ny) == offsetof(Frame, nx) + sizeof(double) * N &&
                  offsetof(Frame, cost) == offsetof(Frame, ny) + sizeof(double) * N &&
                  offsetof(Frame, cid) == offsetof(Frame, nprev) + 12 && sizeof(pp_scene_info) % 4 == 0,
                  "adjacent frame fields");
    if (fio_full) return PP_ERR_STATE;
    {   // the input units in range order, inline where they fit
        int nu = 0;
        for (int r = 0; r < io.n_in; r++) nu += (int)io.in_len[r];
        io.n_inl = 0;
        if (nu <= kFioInline) {
            const uint4* hu = (const uint4*)&h;
            for (int r = 0; r < io.n_in; r++)
                for (uint32_t w = 0; w < io.in_len[r]; w++) io.inl[io.n_inl++] = hu[io.in_off[r] + w];
        }
    }
    void* hdev = nullptr;
    if (hipHostGetDevicePointer(&hdev, DS.frame_host, 0) != hipSuccess) return PP_ERR_HIP;
    io.h_in = (const uint4*)hdev; io.h_out = (uint4*)hdev; io.d_frame = (uint4*)d;
    io.h_flag = (uint32_t*)((char*)hdev + kFlagOff);
    io.seq = ++DS.frame_seq;
#ifdef PP_FRAME_PROF
    const double h1 = fprof_now();
#endif
    int rc = eval_impl(M, &B, &P, &R, device, (void*)st, &io);
#ifdef PP_FRAME_PROF
    const double h2 = fprof_now();
#endif
    if (rc == PP_OK) {
        // the kernel's done word; the stream is polled now and then, so a failed launch or a fault
        // ends the wait with an error
        for (uint64_t spin = 1; *flag != io.seq; spin++) {
            if ((spin & 1023) == 0) {
                const hipError_t e = hipStreamQuery(st);
                if (e == hipSuccess && *flag != io.seq) { rc = PP_ERR_HIP; break; }
                if (e != hipSuccess && e != hipErrorNotReady) { rc = PP_ERR_HIP; break; }
            }
#if defined(__x86_64__) || defined(__i386__)
            __builtin_ia32_pause();
#endif
        }
        std::atomic_thread_fence(std::memory_order_acquire);
#ifdef PP_FRAME_PROF
        const double h3 = fprof_now();
        const volatile uint32_t* fw = flag;
        g_fprof[0] += h1 - h0; g_fprof[1] += h2 - h1; g_fprof[2] += h3 - h2;
        g_fprof[4] += (uint32_t)(fw[5] - fw[4]) / 100.0; g_fprof[5] += (uint32_t)(fw[6] - fw[5]) / 100.0;
        g_fprof[6] += (uint32_t)(fw[7] - fw[6]) / 100.0; g_fprof[7] += 1;
        g_fprof[3] -= h3;             // (done-to-return: the return adds its time)
#endif
    } else if (rc == PP_ERR_STATE) {
        // a launch shape other than the one-launch step (debug shapes, maps beyond the LDS): copies
        if (hipMemcpyAsync(d, &h, sizeof(Frame), hipMemcpyHostToDevice, st) != hipSuccess) return PP_ERR_HIP;
        rc = eval_impl(M, &B, &P, &R, device, (void*)st, nullptr);
        if (rc == PP_OK && (hipMemcpyAsync(&h, d, sizeof(Frame), hipMemcpyDeviceToHost, st) != hipSuccess ||
                            hipStreamSynchronize(st) != hipSuccess))
            rc = PP_ERR_HIP;
    }
    if (rc != PP_OK) return rc;
    DS.plan_table.take_back(hs, 0, nslots);
    *n_out = h.nout;
    for (int i = 0; i < h.nout && i < N; i++) { next_x[i] = h.nx[i]; next_y[i] = h.ny[i]; }
    *target_lane = h.info.target_lane;
#ifdef PP_FRAME_PROF
    g_fprof[3] += fprof_now();
#endif
    return PP_OK;
}

}  // extern "C"

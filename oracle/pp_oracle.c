/*
 * oracle/pp_oracle.c — CPU restatement of the reference's per-frame planning loop.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker for the HIP product path: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * library (carnd-path-planning-project_amd/) never links or calls it.
 *
 * Parity pinning: this restatement is checked bit-for-bit against the reference's own source
 * compiled here (oracle/_ref, built by oracle/Makefile from /root/reference/src) on the golden
 * scene sets in tests/golden/, and its Map::Init output against the reference's DrawLines.ipynb
 * lane0/lane1/lane2 arrays (the only fixture the reference itself holds).
 *
 * Every function cites the reference file:line it follows (Fable3/CarND-Path-Planning-Project).
 * Arithmetic is written in the reference's evaluation order; compile with -ffp-contract=off
 * (x86-64 g++ -O2, the reference's build, never contracts to FMA).
 *
 * Extension beyond the reference (documented in DESIGN.md): the batched candidate grid
 * (lane x target speed), the per-candidate cost and the per-scene argmin. The candidate
 * (planner lane, max_speed) is exactly the reference's single trajectory.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/pp.h"

#define O_PI 3.14159265358979323846 /* helpers.h:33 pi() = M_PI */
#define O_EPS 1e-5                  /* src/main.cpp:24 EPSILON */

typedef struct { double x, y; } P2;

/* Near-threshold census of the acceleration limiter's decisions (src/main.cpp:941, :972; test
 * infrastructure for tests/test_full_batch.py): per calling thread, [0] / [1]
 * decisions taken at :941 / :972, [2] / [3] those whose left side lies within a relative 1e-12 of
 * maximum_acc. ppo_census reads (and optionally clears) the calling thread's counters. */
static _Thread_local long long o_census[4];
static inline void census(int which, double lhs, double mx) {
    o_census[which]++;
    if (fabs(lhs - mx) <= 1e-12 * fabs(mx)) o_census[2 + which]++;
}
void ppo_census(long long* out4, int reset) {
    memcpy(out4, o_census, sizeof o_census);
    if (reset) memset(o_census, 0, sizeof o_census);
}

/* ------------------------------------------------------------------------------------------ */
/* helpers.h geometry                                                                          */
/* ------------------------------------------------------------------------------------------ */
static inline double p_len(P2 p) { return sqrt(p.x * p.x + p.y * p.y); }   /* helpers.h:171 */
static inline double p_lensq(P2 p) { return p.x * p.x + p.y * p.y; }       /* helpers.h:174 */
static inline P2 p_sub(P2 a, P2 b) { P2 r = {a.x - b.x, a.y - b.y}; return r; } /* :165 */
static inline P2 p_add(P2 a, P2 b) { P2 r = {a.x + b.x, a.y + b.y}; return r; } /* :168 */
/* helpers.h:38-40 */
static inline double o_distance(double x1, double y1, double x2, double y2) {
    return sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
}
/* helpers.h:183-186 */
static inline double distsq_pt_pt(P2 p, P2 a) {
    return (p.x - a.x) * (p.x - a.x) + (p.y - a.y) * (p.y - a.y);
}
/* helpers.h:188-249 (quirks: clamp only when rnom < -1; degenerate segment returns 0) */
static double distsq_pt_seg(P2 p, P2 A, P2 B, double* o_rnom, double* o_rdenom, double* o_snom) {
    *o_rnom = 0; *o_rdenom = 1; *o_snom = 0;
    if (A.x == B.x && A.y == B.y) return distsq_pt_pt(A, B);
    const double rdenom = distsq_pt_pt(A, B);
    const double pdx = p.x - A.x, dx = B.x - A.x;
    const double pdy = p.y - A.y, dy = B.y - A.y;
    const double rnom = pdx * dx + pdy * dy;
    *o_rdenom = rdenom;
    const double snom = pdx * dy - pdy * dx;
    *o_snom = snom;
    if (rnom < -1) { *o_rnom = 0; return distsq_pt_pt(p, A); }
    if (rnom > rdenom) { *o_rnom = rdenom; return distsq_pt_pt(p, B); }
    *o_rnom = rnom;
    return snom * snom / rdenom;
}
/* std::min / std::max semantics (NaN handling matters): min(a,b) = (b < a) ? b : a */
static inline double s_min(double a, double b) { return (b < a) ? b : a; }
static inline double s_max(double a, double b) { return (a < b) ? b : a; }

/* ------------------------------------------------------------------------------------------ */
/* Map (src/main.cpp:73-359)                                                                   */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int n;
    P2* ref;
    double *nx, *ny;
    P2 (*lc)[PP_NUM_LANES];
} OMap;

typedef struct {           /* Map::reference_waypoint_id/_ratio (src/main.cpp:132-133), per scene */
    int ref_wp;
    double ratio[PP_NUM_LANES];
} OFrame;

/* src/main.cpp:134-137: (idx + size) % size in size_t arithmetic */
static inline int wpi(const OMap* m, int idx) {
    if (idx >= -m->n) return (idx + m->n) % m->n;
    return (int)(((uint64_t)(int64_t)idx + (uint64_t)m->n) % (uint64_t)m->n);
}
static inline double lane_offset(int lane) { return 4.0 * (lane + 0.5); } /* :84-88 */

/* src/main.cpp:89-131 */
static int omap_init(OMap* m, const double* wx, const double* wy, int n) {
    m->n = n;
    m->ref = (P2*)malloc(sizeof(P2) * n);
    m->nx = (double*)malloc(sizeof(double) * n);
    m->ny = (double*)malloc(sizeof(double) * n);
    m->lc = (P2(*)[PP_NUM_LANES])malloc(sizeof(P2) * PP_NUM_LANES * n);
    if (!m->ref || !m->nx || !m->ny || !m->lc) return -1;
    for (int i = 0; i < n; i++) { m->ref[i].x = wx[i]; m->ref[i].y = wy[i]; }
    for (int i = 0; i < n; i++) {                                       /* :101-109 */
        P2 prev = m->ref[wpi(m, i - 1)];
        P2 delta = p_sub(m->ref[i], prev);
        double dl = p_len(delta);
        m->nx[i] = delta.y / dl;
        m->ny[i] = -delta.x / dl;
    }
    for (int i = 0; i < n; i++) {                                       /* :111-130 */
        int j = wpi(m, i + 1);
        double nx = (m->nx[i] + m->nx[j]) / 2;
        double ny = (m->ny[i] + m->ny[j]) / 2;
        double a_n = atan2(m->ny[i], m->nx[i]);
        double a_avg = atan2(ny, nx);
        double cos_alpha = cos(a_avg - a_n);
        nx /= cos_alpha;
        ny /= cos_alpha;
        for (int r = 0; r < PP_NUM_LANES; r++) {
            double off = lane_offset(r);
            m->lc[i][r].x = m->ref[i].x + nx * off;
            m->lc[i][r].y = m->ref[i].y + ny * off;
        }
    }
    return 0;
}
static void omap_free(OMap* m) { free(m->ref); free(m->nx); free(m->ny); free(m->lc); }

/* src/main.cpp:138-142 */
static inline double lane_len(const OMap* m, int wp, int lane) {
    return p_len(p_sub(m->lc[wpi(m, wp)][lane], m->lc[wpi(m, wp - 1)][lane]));
}

/* src/main.cpp:143-197 */
static void init_reference_waypoint(const OMap* m, OFrame* f, double x, double y) {
    int closest = 0;
    P2 p = {x, y};
    double cd = p_lensq(p_sub(m->ref[0], p));
    for (int i = 1; i < m->n; i++) {
        double d = p_lensq(p_sub(m->ref[i], p));
        if (d < cd) { closest = i; cd = d; }
    }
    double rnom, snom, rdenom, dref[2];
    for (int k = 0; k < 2; k++)
        dref[k] = distsq_pt_seg(p, m->ref[wpi(m, closest + k - 1)], m->ref[wpi(m, closest + k)],
                                &rnom, &rdenom, &snom);
    if (dref[1] < dref[0]) {
        closest++;
    } else if (dref[1] == dref[0]) {
        int a = wpi(m, closest - 1), b = wpi(m, closest);
        P2 an = {(m->nx[a] + m->nx[b]) / 2, (m->ny[a] + m->ny[b]) / 2};
        P2 dp = p_sub(p, m->ref[b]);
        double dotp = an.x * dp.x + an.y * dp.y;
        if (dotp > 0) closest++;
    }
    f->ref_wp = closest;
    for (int lane = 0; lane < PP_NUM_LANES; lane++) {
        distsq_pt_seg(p, m->lc[wpi(m, closest - 1)][lane], m->lc[wpi(m, closest)][lane], &rnom,
                      &rdenom, &snom);
        f->ratio[lane] = rnom / rdenom;
    }
}

/* src/main.cpp:199-275. Returns found_any. The walk is bounded (the reference's terminates by
 * strict improvement); the bound is never reached on finite inputs. */
static int lane_matching(const OMap* m, const OFrame* f, double x, double y, double* out_s,
                         double* out_d, int* out_lane, int* out_next_wp) {
    int dir = 0;
    P2 p = {x, y};
    int stop = 0;
    int cur = f->ref_wp;
    double sum_s[PP_NUM_LANES] = {0};
    double s_ratio[PP_NUM_LANES];
    for (int i = 0; i < PP_NUM_LANES; i++) s_ratio[i] = f->ratio[i];
    double best = 1000 * 1000;
    int found = 0;
    for (int it = 0; it < 4 * m->n + 8; it++) {
        double rnom, snom, rdenom;
        int improved = 0;
        for (int lane = 0; lane < PP_NUM_LANES; lane++) {
            double dsq = distsq_pt_seg(p, m->lc[wpi(m, cur - 1)][lane], m->lc[wpi(m, cur)][lane],
                                       &rnom, &rdenom, &snom);
            if (dsq < best) {
                best = dsq;
                improved = 1;
                found = 1;
                double ratio_from_start = rnom / rdenom;
                double r_mod = ratio_from_start - s_ratio[lane];
                double seg_len = lane_len(m, cur, lane);
                *out_s = sum_s[lane] + seg_len * r_mod;
                double d = sqrt(dsq);
                if (snom < 0) d = -d;
                *out_d = d + lane_offset(lane);
                *out_lane = lane;
                if (out_next_wp) *out_next_wp = cur;
            }
            if (rnom == 0) {
                if (dir == 1) stop = 1;
                dir = -1;
            } else if (rnom == rdenom) {
                if (dir == -1) stop = 1;
                dir = 1;
            } else {
                stop = 1;
            }
        }
        if (!improved || stop) break;
        if (dir > 0) {
            for (int lane = 0; lane < PP_NUM_LANES; lane++) {
                sum_s[lane] += (1 - s_ratio[lane]) * lane_len(m, cur, lane);
                s_ratio[lane] = 0;
            }
            cur++;
        } else {
            for (int lane = 0; lane < PP_NUM_LANES; lane++) {
                sum_s[lane] -= s_ratio[lane] * lane_len(m, cur, lane);
                s_ratio[lane] = 1;
            }
            cur--;
        }
    }
    return found;
}

/* src/main.cpp:277-328. *ok = 0 if the (bounded) walk did not terminate (NaN s). */
static P2 get_lane_pos(const OMap* m, const OFrame* f, double s, int lane, int* ok) {
    double ratio = f->ratio[lane];
    int wp = f->ref_wp;
    P2 nxt = {0, 0}, prv = {0, 0};
    double dest = 0;
    *ok = 0;
    for (int it = 0; it < 4 * m->n + 8; it++) {
        nxt = m->lc[wpi(m, wp)][lane];
        prv = m->lc[wpi(m, wp - 1)][lane];
        double wl = p_len(p_sub(nxt, prv));
        if (s > 0) {
            double rem = wl * (1 - ratio);
            if (s <= rem) { dest = 1 - (rem - s) / wl; *ok = 1; break; }
            s -= rem;
            ratio = 0;
            wp++;
        } else {
            double rem = wl * ratio;
            if (-s <= rem) { dest = (rem + s) / wl; *ok = 1; break; }
            s += rem;
            ratio = 1;
            wp--;
        }
    }
    P2 r;
    r.x = nxt.x * dest + prv.x * (1 - dest);
    r.y = nxt.y * dest + prv.y * (1 - dest);
    return r;
}

/* src/main.cpp:330-358 */
static void project_speed(const OMap* m, P2 v, int next_wp, double* vs, double* vd) {
    double rnom, snom, rdenom;
    P2 w = p_sub(m->ref[wpi(m, next_wp)], m->ref[wpi(m, next_wp - 1)]);
    double svl = p_len(v);
    if (svl < O_EPS) {
        *vs = svl;
        *vd = 0;
    } else {
        double wvl = p_len(w);
        w.x *= svl / wvl;
        w.y *= svl / wvl;
        double sign = 1.0;
        if (w.x * v.x + w.y * v.y < 0) { v.x *= -1; v.y *= -1; sign = -1; }
        P2 zero = {0, 0};
        distsq_pt_seg(v, zero, w, &rnom, &rdenom, &snom);
        *vs = (rnom / rdenom) * svl * sign;
        *vd = (snom / rdenom) * svl * sign;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Car (src/main.cpp:51-71)                                                                     */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int id;
    double x, y, vx, vy, s, d, vs, vd;
    int lane;
} OCar;

/* ------------------------------------------------------------------------------------------ */
/* LaneChangePlanner::calculate_target_lane (src/main.cpp:364-485)                              */
/* ------------------------------------------------------------------------------------------ */
static int calc_target_lane(const pp_params* P, const OCar* cars, int nc, int ego_lane,
                            int target_lane, double ego_s, double ego_vs, double dt0,
                            double* score_out, int* open_mask, int* jump_rule) {
    double lane_speed[PP_NUM_LANES], next_s[PP_NUM_LANES];
    int open[PP_NUM_LANES];
    for (int i = 0; i < PP_NUM_LANES; i++) { lane_speed[i] = P->max_speed; next_s[i] = 1000; open[i] = 1; }
    for (int k = 0; k < nc; k++) {
        const OCar* o = &cars[k];
        int lane = o->lane;
        double s = o->s + o->vs * dt0;
        if (s > ego_s) {
            if (s < next_s[lane]) {
                next_s[lane] = s;
                if (s - ego_s < 200) {
                    int speed = (int)o->vs;
                    if (speed > P->max_speed) speed = (int)P->max_speed;
                    if (s - ego_s > 100)
                        speed = (int)(speed + (P->max_speed - speed) * (s - ego_s - 100) / (200.0 - 100.0));
                    lane_speed[lane] = speed;
                }
            }
        }
        double add = 2;
        if (target_lane == lane) add = 0;
        double min_dist = P->car_length + P->safety_distance + add;
        if (fabs(ego_s - s) < min_dist) open[lane] = 0;
        if (s > ego_s && o->vs < ego_vs) {
            double car_dist = s - ego_s - P->car_length - P->safety_distance - add;
            double sd = ego_vs - o->vs;
            double dtm = sd / P->relaxed_acc;
            double ddist = ego_vs * dtm - sd / 2 * dtm;
            if (car_dist < ddist) open[lane] = 0;
        }
        if (s < ego_s && o->vs > ego_vs && s + 50 > ego_s) {
            double car_dist = ego_s - s - P->car_length - P->safety_distance - add;
            double sd = o->vs - ego_vs;
            double dtm = sd / P->relaxed_acc;
            if (target_lane == ego_lane) dtm += 2;
            double md = sd * dtm;
            if (car_dist < md) open[lane] = 0;
        }
    }
    int best_lane = ego_lane;
    double best_score = 0;
    for (int lane = 0; lane < PP_NUM_LANES; lane++) {
        score_out[lane] = 0;
        if (lane != ego_lane && !open[lane]) continue;
        double speed_score = s_min(lane_speed[lane] / P->max_speed, 1.0);
        double distance_score = 1 - fabs((double)(target_lane - lane)) / 2;
        double free_score = s_min(1.0, next_s[lane] / 100);
        double total = speed_score + distance_score / 2 + free_score;
        score_out[lane] = total;
        if (total > best_score) { best_score = total; best_lane = lane; }
    }
    *open_mask = 0;
    for (int lane = 0; lane < PP_NUM_LANES; lane++) *open_mask |= open[lane] << lane;
    *jump_rule = 0;
    if (abs(ego_lane - best_lane) > 1) {
        int nl = best_lane > ego_lane ? ego_lane + 1 : ego_lane - 1;
        target_lane = open[nl] ? nl : ego_lane;
        *jump_rule = 1;
    } else {
        target_lane = best_lane;
    }
    return target_lane;
}

/* ------------------------------------------------------------------------------------------ */
/* SpeedController (src/main.cpp:488-548)                                                      */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double start, target, ttime, shift; } OSC;

static inline double sc_get_speed(const OSC* c, double t) {   /* :503-512 */
    t -= c->shift;
    if (t < 0) t = 0;
    if (t > c->ttime) return c->target;
    return c->start + (c->target - c->start) * t / c->ttime;
}
static inline void sc_add_limit(OSC* c, double nts, double ntt) {   /* :513-533 */
    double tm = s_max(c->ttime, 0.02);
    double ntm = s_max(ntt, 0.02);
    double cg = (c->target - c->start) / tm;
    double ng = (nts - c->start) / ntm;
    if (ng < cg) { c->target = nts; c->ttime = ntt; }
}
static inline void sc_override(OSC* c, double t, double speed) {   /* :534-547 */
    if (t > c->ttime) return;
    if (fabs(c->target - c->start) < O_EPS) return;
    double mt = c->ttime * (speed - c->start) / (c->target - c->start);
    c->shift = t - mt;
}

/* ------------------------------------------------------------------------------------------ */
/* LimitSpeed::calculate (src/main.cpp:1052-1151). Returns code: 0 FREEFLOW 1 BRAKE 2 MAXBRAKE  */
/* 3 ADJUST 4 KEEP; *collision set when the gap was negative.                                   */
/* ------------------------------------------------------------------------------------------ */
static int limit_speed(const pp_params* P, const OCar* fc, double next_s, double ego_s,
                       double ego_speed, double ego_acc, int in_lane, double* ts, double* tt,
                       int* collision) {
    int code = 0, can_acc = 1;
    *ts = P->max_speed;
    *tt = fabs(ego_speed - P->max_speed) / P->relaxed_acc;
    double fcd = next_s - ego_s - P->car_length;
    *collision = 0;
    if (fcd < 0) { fcd = 0; *collision = 1; }
    double fcs = sqrt(fc->vx * fc->vx + fc->vy * fc->vy);
    if (ego_speed > fcs) {
        double acc = P->relaxed_acc;
        if (ego_acc < 0) acc = P->min_relaxed_acc_while_braking;
        double dv = ego_speed - fcs;
        double dt = dv / acc;
        double dd = ego_speed * dt - dv / 2 * dt;
        double max_dist = fcd - P->safety_distance;
        if (dd > max_dist) {
            *ts = fcs;
            *tt = max_dist / (ego_speed - dv / 2);
            if (*tt < O_EPS || dv / *tt > P->maximum_acc) { code = 2; *tt = dv / P->maximum_acc; }
            else code = 1;
            can_acc = 0;
        }
    }
    if (can_acc && in_lane) {
        double excess = ego_s + P->car_length + P->keep_distance - next_s;
        double t_opt = s_min(1.0, fabs(excess) / 1.0);
        if (ego_s + P->car_length + P->keep_distance > next_s) {
            *ts = fcs - excess / t_opt;
            *tt = t_opt;
            double mt = fabs(*ts - ego_speed) / P->relaxed_acc;   /* maximize_acc :1059-1067 */
            if (*tt < mt) *tt = mt;
            code = 3;
        } else if (ego_s + P->car_length + P->keep_distance + P->keep_distance_leeway > next_s) {
            *ts = fcs;
            *tt = 1.0;
            double mt = fabs(*ts - ego_speed) / P->relaxed_acc;
            if (*tt < mt) *tt = mt;
            code = 4;
        }
    }
    return code;
}

/* ------------------------------------------------------------------------------------------ */
/* tk::spline (src/spline.h:284-396): natural cubic spline, band LU without pivoting           */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int n;
    double x[PP_MAX_KNOTS], y[PP_MAX_KNOTS], a[PP_MAX_KNOTS], b[PP_MAX_KNOTS], c[PP_MAX_KNOTS];
    double b0, c0;
} OSpline;

static void spline_set_points(OSpline* sp, const double* x, const double* y, int n) {
    /* band_matrix(n,1,1): up0 = diag, up1 = upper, lo0 = saved_diag, lo1 = lower (spline.h:130-184) */
    double up0[PP_MAX_KNOTS] = {0}, up1[PP_MAX_KNOTS] = {0}, lo0[PP_MAX_KNOTS] = {0}, lo1[PP_MAX_KNOTS] = {0};
    double rhs[PP_MAX_KNOTS] = {0}, yy[PP_MAX_KNOTS], bb[PP_MAX_KNOTS];
    sp->n = n;
    for (int i = 0; i < n; i++) { sp->x[i] = x[i]; sp->y[i] = y[i]; }
    for (int i = 1; i < n - 1; i++) {                                   /* spline.h:302-307 */
        lo1[i] = 1.0 / 3.0 * (x[i] - x[i - 1]);
        up0[i] = 2.0 / 3.0 * (x[i + 1] - x[i - 1]);
        up1[i] = 1.0 / 3.0 * (x[i + 1] - x[i]);
        rhs[i] = (y[i + 1] - y[i]) / (x[i + 1] - x[i]) - (y[i] - y[i - 1]) / (x[i] - x[i - 1]);
    }
    up0[0] = 2.0; up1[0] = 0.0; rhs[0] = 0.0;                           /* :309-313 */
    up0[n - 1] = 2.0; lo1[n - 1] = 0.0; rhs[n - 1] = 0.0;               /* :323-327 */
    /* lu_decompose (spline.h:187-220) */
    for (int i = 0; i < n; i++) {
        lo0[i] = 1.0 / up0[i];
        if (i > 0) lo1[i] *= lo0[i];
        up0[i] *= lo0[i];
        if (i < n - 1) up1[i] *= lo0[i];
        up0[i] = 1.0;
    }
    for (int k = 0; k < n - 1; k++) {
        double xx = -lo1[k + 1] / up0[k];
        lo1[k + 1] = -xx;
        up0[k + 1] = up0[k + 1] + xx * up1[k];
    }
    /* l_solve (:222-235), r_solve (:237-250) */
    for (int i = 0; i < n; i++) {
        double sum = 0;
        if (i > 0) sum += lo1[i] * yy[i - 1];
        yy[i] = (rhs[i] * lo0[i]) - sum;
    }
    for (int i = n - 1; i >= 0; i--) {
        double sum = 0;
        if (i < n - 1) sum += up1[i] * bb[i + 1];
        bb[i] = (yy[i] - sum) / up0[i];
    }
    for (int i = 0; i < n; i++) sp->b[i] = bb[i];
    for (int i = 0; i < n - 1; i++) {                                   /* :345-349 */
        sp->a[i] = 1.0 / 3.0 * (bb[i + 1] - bb[i]) / (x[i + 1] - x[i]);
        sp->c[i] = (y[i + 1] - y[i]) / (x[i + 1] - x[i]) - 1.0 / 3.0 * (2.0 * bb[i] + bb[i + 1]) * (x[i + 1] - x[i]);
    }
    sp->b0 = sp->b[0];                                                  /* :362-372 */
    sp->c0 = sp->c[0];
    double h = x[n - 1] - x[n - 2];
    sp->a[n - 1] = 0.0;
    sp->c[n - 1] = 3.0 * sp->a[n - 2] * h * h + 2.0 * sp->b[n - 2] * h + sp->c[n - 2];
}

static double spline_eval(const OSpline* sp, double x) {               /* spline.h:375-396 */
    int n = sp->n;
    int lb = 0;                       /* std::lower_bound: first i with !(x_i < x) */
    while (lb < n && sp->x[lb] < x) lb++;
    int idx = lb - 1 > 0 ? lb - 1 : 0;
    double h = x - sp->x[idx];
    if (x < sp->x[0]) return (sp->b0 * h + sp->c0) * h + sp->y[0];
    if (x > sp->x[n - 1]) return (sp->b[n - 1] * h + sp->c[n - 1]) * h + sp->y[n - 1];
    return ((sp->a[idx] * h + sp->b[idx]) * h + sp->c[idx]) * h + sp->y[idx];
}

/* ------------------------------------------------------------------------------------------ */
/* Scene preparation: onMessage compute body (src/main.cpp:1254-1438)                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int K;                           /* previous points kept: 10 or 0 (:1261)                   */
    P2 prev[PP_PREV_KEEP];
    double ego_x, ego_y, yaw, ego_speed, ego_acc, dt0;
    OFrame fr;
    double ego_s, ego_d, ego_vs, ego_vd;
    int ego_lane, T, open_mask;
    double score[PP_NUM_LANES];
    /* follow limits: in-lane (:1425-1431) and per candidate lane (:1432-1438) */
    int has_in;
    double in_ts, in_tt;
    int has_l[PP_NUM_LANES];
    double l_ts[PP_NUM_LANES], l_tt[PP_NUM_LANES];
    int nmatched, in_id;
    uint32_t status;
} OPrep;

static const uint32_t limit_flag[5] = {0, PP_ST_BRAKE, PP_ST_MAXBRAKE, PP_ST_ADJUST, PP_ST_KEEP};

/* Monte-Carlo sensor noise (build extension, include/pp.h pp_params / pp_mc_gauss): Philox4x32-10
 * block keyed by the seed, counter {scene, (draw * PP_NOISE_CAR_STRIDE + car) * 4 + q, 0x4D43}; Irwin-Hall of its
 * four 32-bit uniforms scaled to unit variance. */
static double mc_gauss(uint64_t seed, uint64_t scene, int draw, int car, int q) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)scene, (uint32_t)(scene >> 32), (uint32_t)((draw * PP_NOISE_CAR_STRIDE + car) * 4 + q), 0x4D43u};
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0], p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ ctr[1] ^ key[0];
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ ctr[3] ^ key[1];
        ctr[0] = n0; ctr[1] = (uint32_t)p1; ctr[2] = n2; ctr[3] = (uint32_t)p0;
        key[0] += 0x9E3779B9u;
        key[1] += 0xBB67AE85u;
    }
    const double k = 1.0 / 4294967296.0;
    double a = ((double)ctr[0] + 0.5) * k;
    a += ((double)ctr[1] + 0.5) * k;
    a += ((double)ctr[2] + 0.5) * k;
    a += ((double)ctr[3] + 0.5) * k;
    return (a - 2.0) * 1.7320508075688772;
}

double ppo_mc_gauss(uint64_t seed, int64_t scene, int draw, int car, int q) {
    return mc_gauss(seed, (uint64_t)scene, draw, car, q);
}

/* draw > 0: the sensor-fusion cars carry Monte-Carlo noise (P->n_draws) */
static void prep_scene(const OMap* m, const pp_params* P, const pp_scene_batch* in, int64_t s,
                       int draw, OPrep* pr) {
    const int64_t S = in->n_scenes;
    memset(pr, 0, sizeof(*pr));
    pr->ego_x = in->ego_x[s];
    pr->ego_y = in->ego_y[s];
    pr->yaw = in->ego_yaw_deg[s];
    double ego_speed = in->ego_speed_mph[s];
    ego_speed /= 2.237;                                                 /* :1239 */
    double ego_acc = 0;
    P2 esv = {0, 0};
    pr->dt0 = 0;
    pr->K = 0;
    if (in->n_prev[s] >= PP_PREV_KEEP) {                                /* :1261-1282 */
        pr->K = PP_PREV_KEEP;
        for (int i = 0; i < PP_PREV_KEEP; i++) {
            pr->prev[i].x = in->prev_x[(int64_t)i * S + s];
            pr->prev[i].y = in->prev_y[(int64_t)i * S + s];
        }
        double v2 = p_len(p_sub(pr->prev[8], pr->prev[7]));
        esv = p_sub(pr->prev[9], pr->prev[8]);
        double v3 = p_len(esv);
        ego_acc = (v3 - v2) * 50;
        ego_speed = v3 * 50;
        esv.x *= 50;
        esv.y *= 50;
        pr->ego_x = pr->prev[9].x;
        pr->ego_y = pr->prev[9].y;
        pr->dt0 = PP_PREV_KEEP / 50.0;
    }
    init_reference_waypoint(m, &pr->fr, pr->ego_x, pr->ego_y);          /* :1299 */
    double ego_s = 0, ego_d = 0;
    int ego_lane = 0;
    if (!lane_matching(m, &pr->fr, pr->ego_x, pr->ego_y, &ego_s, &ego_d, &ego_lane, NULL)) {
        ego_s = ego_d = 0;                                              /* :1302-1307 */
        ego_lane = 0;
        pr->status |= PP_ST_EGO_UNMATCHED;
    }
    double ego_vs, ego_vd;
    project_speed(m, esv, pr->fr.ref_wp, &ego_vs, &ego_vd);            /* :1313 */
    if (ego_acc > P->maximum_acc) ego_acc = P->maximum_acc;             /* :1319-1320 */
    if (ego_acc < -P->maximum_acc) ego_acc = -P->maximum_acc;

    OCar cars[PP_MAX_CARS];                                             /* :1325-1350 */
    int nc = 0;
    int ncar = in->n_cars[s];
    if (ncar > in->car_stride) ncar = in->car_stride;
    /* with a car table (the reference's persistent std::map, :1194): the tab_slots slots in order
     * (ascending id, include/pp.h), each car reported this frame (re-matched: slot overwritten, or
     * erased, :1329-1348) or taken from its stale slot; without one: the frame's rows in
     * (ascending id) order */
    const int tab = in->tab_valid != NULL;
    const int iters = tab ? in->tab_slots : ncar;
    int p = 0;
    for (int it = 0; it < iters; it++) {
        int row = it;
        const int64_t tix = (int64_t)it * S + s;
        const int sid = tab ? (in->tab_id ? in->tab_id[tix] : it) : 0;
        if (tab) {
            while (p < ncar && in->car_id[(int64_t)p * S + s] < sid) p++;
            row = (p < ncar && in->car_id[(int64_t)p * S + s] == sid) ? p++ : -1;
        }
        OCar c;
        memset(&c, 0, sizeof(c));
        if (row >= 0) {
            int64_t ix = (int64_t)row * S + s;
            c.id = in->car_id[ix];
            c.x = in->car_x[ix];
            c.y = in->car_y[ix];
            c.vx = in->car_vx[ix];
            c.vy = in->car_vy[ix];
            if (draw > 0) {
                const uint64_t gs = (uint64_t)(P->noise_first_scene + s);
                c.x += P->noise_pos_sigma * mc_gauss(P->noise_seed, gs, draw, row, 0);
                c.y += P->noise_pos_sigma * mc_gauss(P->noise_seed, gs, draw, row, 1);
                c.vx += P->noise_vel_sigma * mc_gauss(P->noise_seed, gs, draw, row, 2);
                c.vy += P->noise_vel_sigma * mc_gauss(P->noise_seed, gs, draw, row, 3);
            }
            int nwp = 0;
            if (!lane_matching(m, &pr->fr, c.x, c.y, &c.s, &c.d, &c.lane, &nwp)) {
                pr->status |= PP_ST_CAR_UNMATCHED;
                if (tab) in->tab_valid[tix] = 0;
                continue;
            }
            P2 v = {c.vx, c.vy};
            project_speed(m, v, nwp, &c.vs, &c.vd);
            if (tab) {
                in->tab_valid[tix] = 1; in->tab_lane[tix] = c.lane;
                in->tab_s[tix] = c.s; in->tab_d[tix] = c.d; in->tab_vs[tix] = c.vs; in->tab_vd[tix] = c.vd;
                in->tab_vx[tix] = c.vx; in->tab_vy[tix] = c.vy;
            }
        } else {
            if (!in->tab_valid[tix]) continue;
            c.id = sid;
            c.lane = in->tab_lane[tix];
            c.s = in->tab_s[tix]; c.d = in->tab_d[tix]; c.vs = in->tab_vs[tix]; c.vd = in->tab_vd[tix];
            c.vx = in->tab_vx[tix]; c.vy = in->tab_vy[tix];
        }
        cars[nc++] = c;
    }
    pr->nmatched = nc;
    int jump = 0;
    int T = calc_target_lane(P, cars, nc, ego_lane, in->prev_target_lane[s], ego_s, ego_vs,
                             pr->dt0, pr->score, &pr->open_mask, &jump);   /* :1352-1356 */
    if (jump) pr->status |= PP_ST_JUMP_RULE;
    if (pr->open_mask != (1 << PP_NUM_LANES) - 1) pr->status |= PP_ST_LANE_CLOSED;
    if (T != ego_lane) {                                                /* :1358-1369 */
        double dtl = lane_offset(T);
        double diff = fabs(ego_vd * 1.0 + ego_d - dtl);
        if (diff > 6.0) { T = ego_lane; pr->status |= PP_ST_TOO_FAR; }
    }
    /* follow-car selection (:1383-1411), for the in-lane car and for every candidate lane */
    /* the reference tracks the chosen car by its id with -1 as "none" (:1383-1411): a car whose id
     * is -1 is chosen and still reads as none, so the next qualifying car replaces it and no
     * limit follows it; the ids are what :1411 compares */
    int in_id = -1, in_k = -1;
    double in_s = 0;
    int t_id[PP_NUM_LANES], tk[PP_NUM_LANES];
    double ts_[PP_NUM_LANES];
    for (int L = 0; L < PP_NUM_LANES; L++) { t_id[L] = -1; tk[L] = -1; ts_[L] = 0; }
    for (int k = 0; k < nc; k++) {
        double s0 = cars[k].s + cars[k].vs * pr->dt0;
        double d0 = cars[k].d + cars[k].vd * pr->dt0;
        if (s0 > ego_s && fabs(d0 - ego_d) < 3) {
            if (in_id == -1 || in_s > s0) { in_id = cars[k].id; in_k = k; in_s = s0; }
        }
        for (int L = 0; L < PP_NUM_LANES; L++) {
            if (s0 >= ego_s - P->car_length - P->safety_distance && fabs(d0 - lane_offset(L)) < 3) {
                if (t_id[L] == -1 || ts_[L] > s0) { t_id[L] = cars[k].id; tk[L] = k; ts_[L] = s0; }
            }
        }
    }
    if (in_id == -1) in_k = -1;
    pr->in_id = in_id;
    int col = 0, code;
    if (in_k >= 0) {                                                    /* :1425-1431 */
        pr->has_in = 1;
        code = limit_speed(P, &cars[in_k], in_s, ego_s, ego_speed, ego_acc, 1, &pr->in_ts, &pr->in_tt, &col);
        pr->status |= limit_flag[code] | (col ? PP_ST_COLLISION : 0);
    }
    for (int L = 0; L < PP_NUM_LANES; L++) {                            /* :1411, 1432-1438 */
        if (t_id[L] == -1 || t_id[L] == in_id) tk[L] = -1;
        pr->has_l[L] = tk[L] >= 0;
        if (tk[L] >= 0) {
            code = limit_speed(P, &cars[tk[L]], ts_[L], ego_s, ego_speed, ego_acc, 0, &pr->l_ts[L], &pr->l_tt[L], &col);
            pr->status |= limit_flag[code] | (col ? PP_ST_COLLISION : 0);
        }
    }
    pr->ego_speed = ego_speed;
    pr->ego_acc = ego_acc;
    pr->ego_s = ego_s;
    pr->ego_d = ego_d;
    pr->ego_vs = ego_vs;
    pr->ego_vd = ego_vd;
    pr->ego_lane = ego_lane;
    pr->T = T;
}

/* candidate speed grid (build extension): k = 0 -> max_speed */
static inline double cand_speed(const pp_params* P, double ego_speed, int k) {
    if (k == 0) return P->max_speed;
    double v = ego_speed + P->speed_offsets[k - 1];
    if (v < 0) v = 0;
    if (v > P->max_speed) v = P->max_speed;
    return v;
}

/* ------------------------------------------------------------------------------------------ */
/* TrajectoryBuilder::build (src/main.cpp:565-1049) for candidate lane L + speed controller sc */
/* Writes generated points (after the K kept ones) into gx/gy; returns their count.            */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double acc_sum, travelled; int fallback, trunc, override_hit, curv_hit, walk_fail; } OStats;

static int build_traj(const OMap* m, const pp_params* P, const OPrep* pr, int L, OSC sc,
                      int Npts, double* gx, double* gy, OStats* st) {
    memset(st, 0, sizeof(*st));
    const int K = pr->K;
    double pos_x, pos_y, angle;
    if (K == 0) {                                                       /* :583-610 */
        pos_x = pr->ego_x; pos_y = pr->ego_y;
        angle = pr->yaw * O_PI / 180;
    } else {
        pos_x = pr->prev[K - 1].x; pos_y = pr->prev[K - 1].y;
        if (K == 1) angle = pr->yaw * O_PI / 180;
        else {
            double px2 = pr->prev[K - 2].x, py2 = pr->prev[K - 2].y;
            P2 v = {pos_x - px2, pos_y - py2};
            if (p_lensq(v) < O_EPS) angle = pr->yaw * O_PI / 180;
            else angle = atan2(pos_y - py2, pos_x - px2);
        }
    }
    /* control points (:638-768) */
    P2 cp[6];
    int ncp = 0;
    double total_dist = 0;
    cp[ncp++] = (P2){pos_x, pos_y};
    double min_cpd = sc.start * 1;
    min_cpd = s_max(min_cpd, 5.0);
    double d_diff = lane_offset(L) - pr->ego_d;
    double ego_vd = pr->ego_vd;
    double d_acc = 4;
    int slow = 0;
    double lst = 2.0;
    if ((ego_vd < 0) == (d_diff < 0)) {
        double dmax = ego_vd * ego_vd / d_acc / 2;
        if (dmax > fabs(d_diff)) { slow = 1; lst = fabs(ego_vd) / d_acc; }
    }
    if (!slow) {
        double rel = ego_vd;
        if (d_diff < 0) rel *= -1;
        double add = fabs(d_diff);
        double peak = sqrt(add * d_acc + rel * rel / 2);
        lst = (peak * 2 - rel) / d_acc;
    }
    double dist = sc.start * lst;
    if (dist < 10.0) dist = 10.0;
    if (dist > 50) dist = 50;
    double cps = dist;
    for (int i = 0; i < 5; i++) {
        int ok;
        P2 np = get_lane_pos(m, &pr->fr, cps, L, &ok);
        if (!ok) st->walk_fail = 1;
        P2 pp = cp[ncp - 1];
        total_dist += o_distance(pp.x, pp.y, np.x, np.y);
        cp[ncp++] = np;
        if (total_dist > 50 && ncp > 2) break;
        cps += min_cpd;
    }
    /* local frame (:786-831) */
    double ca = cos(-angle), sa = sin(-angle);
    P2 center = {pos_x, pos_y};
    for (int i = 0; i < ncp; i++) {
        P2 p = p_sub(cp[i], center);
        double tx = p.x * ca - p.y * sa;
        double ty = p.x * sa + p.y * ca;
        cp[i].x = tx; cp[i].y = ty;
    }
    double kx[PP_MAX_KNOTS], ky[PP_MAX_KNOTS];
    int nk = 0;
    for (int i = 0; i < K - 1; i++) {
        P2 t = p_sub(pr->prev[i], center);
        kx[nk] = t.x * ca - t.y * sa;
        ky[nk] = t.x * sa + t.y * ca;
        nk++;
    }
    int min_cp_count = nk;
    pos_x = 0; pos_y = 0;
    double tangle = angle;
    ca = cos(tangle); sa = sin(tangle);
    for (int i = 0; i < ncp; i++) { kx[nk] = cp[i].x; ky[nk] = cp[i].y; nk++; }
    for (int i = 1; i < nk; i++) {                                      /* :833-843 */
        if (kx[i] <= kx[i - 1]) { nk = i; st->trunc = 1; break; }
    }
    double cur_t = 0.02;
    int ng = 0;
    const int room = Npts - K;
    if (nk < 3 || nk <= min_cp_count || fabs(pr->ego_d) > 20) {         /* :848-901 fallback */
        st->fallback = 1;
        double speed = sc_get_speed(&sc, cur_t);
        double cang = 0;
        int nc = 1;
        while (ng < room && nc < ncp) {
            double dstep = speed / 50;
            P2 nd = p_sub(cp[nc], (P2){pos_x, pos_y});
            double cpd = p_len(nd);
            if (cpd < 5) { nc++; continue; }
            cur_t += 0.02;
            double nca = atan2(nd.y, nd.x);
            double adiff = fmod(nca - cang + 3 * O_PI, 2 * O_PI) - O_PI;
            double min_radius = s_max(10.0, speed * speed / 4);
            double rps = speed / min_radius;
            double mas = rps / 50;
            if (fabs(adiff) > mas) {
                if (adiff > 0) cang += mas; else cang -= mas;
            } else {
                cang += adiff;
            }
            pos_x += cos(cang) * dstep;
            pos_y += sin(cang) * dstep;
            double tx = pos_x * ca - pos_y * sa;
            double ty = pos_x * sa + pos_y * ca;
            gx[ng] = tx + center.x;
            gy[ng] = ty + center.y;
            ng++;
            st->travelled += dstep;
        }
        return ng;
    }
    OSpline sp;
    spline_set_points(&sp, kx, ky, nk);                                 /* :904 */
    double arg = 0, prev_speed = sc.start, prev_angle = 0;
    while (arg < 50 && ng < room) {                                     /* :911-1040 */
        double speed = sc_get_speed(&sc, cur_t);
        double dstep = speed / 50;
        double yv = spline_eval(&sp, arg + dstep);
        double x = arg + dstep;
        double y = yv;
        double d = o_distance(pos_x, pos_y, x, y);
        double acc = fabs(speed - prev_speed) * 50;
        double astep = atan2(y - pos_y, x - pos_x);
        double adiff = fmod(astep - prev_angle + 3 * O_PI, 2 * O_PI) - O_PI;
        double cacc = speed * 50 * fabs(adiff);
        double eff_c = cacc;
        census(0, acc + cacc, P->maximum_acc);
        if (acc + cacc > P->maximum_acc) {
            if (speed > prev_speed) {
                double na = P->maximum_acc - cacc;
                if (na < 0) na = 0;
                double ns = prev_speed + na / 50;
                sc_override(&sc, cur_t, ns);
                speed = ns;
                sc.ttime += 0.02;
                dstep = speed / 50;
                acc = na;
                st->override_hit = 1;
            }
            census(1, acc + cacc, P->maximum_acc);
            if (acc + cacc > P->maximum_acc) {
                double nc = P->maximum_acc - acc;
                if (nc < 0) nc = 0;
                double nad = nc / speed / 50;
                if (adiff < 0) nad *= -1;
                double rot = nad - adiff;
                double tpx = pos_x * ca - pos_y * sa;
                double tpy = pos_x * sa + pos_y * ca;
                tpx = tpx + center.x;
                tpy = tpy + center.y;
                double vx = center.x - tpx, vy = center.y - tpy;
                double rvx = vx * cos(rot) - vy * sin(rot);
                double rvy = vx * sin(rot) + vy * cos(rot);
                center.x = tpx + rvx;
                center.y = tpy + rvy;
                tangle += rot;
                ca = cos(tangle);
                sa = sin(tangle);
                eff_c = nc;
                st->curv_hit = 1;
            }
        }
        cur_t += 0.02;
        prev_speed = speed;
        prev_angle = astep;
        double sp_step = (x - pos_x) * dstep / d;
        pos_y += (y - pos_y) * dstep / d;
        arg += sp_step;
        pos_x += sp_step;
        double tx = pos_x * ca - pos_y * sa;
        double ty = pos_x * sa + pos_y * ca;
        gx[ng] = tx + center.x;
        gy[ng] = ty + center.y;
        ng++;
        st->acc_sum += acc + eff_c;
        st->travelled += dstep;
    }
    return ng;
}

/* per-candidate cost (build extension). Identical formula in the HIP kernel. */
static double cand_cost(const pp_params* P, const OPrep* pr, int L, double v, int ng,
                        const OStats* st, int* is_nan) {
    double acc_mean = ng > 0 ? st->acc_sum / ng : 0.0;
    double ideal = (P->n_points - pr->K) * P->max_speed / 50;
    double deficit = 1.0 - st->travelled / ideal;
    double J = (2.5 - pr->score[L]) + acc_mean / P->maximum_acc + deficit + (st->fallback ? 1.0 : 0.0);
    *is_nan = 0;
    if (!(J == J) || st->walk_fail) { J = 999.0; *is_nan = 1; }
    if (J > 999.0) J = 999.0;
    if (J < 0.0) J = 0.0;
    if (P->cost_mode == PP_COST_REFERENCE) {
        if (L != pr->T) J += 1e6;
        if (v != P->max_speed) J += 1e3;
    } else {
        if (!((pr->open_mask >> L) & 1) && L != pr->ego_lane) J += 10.0;
    }
    return J;
}

static OSC make_sc(const pp_params* P, const OPrep* pr, int L, double v) {
    OSC sc;                                         /* SpeedController ctor :495-502, target v */
    sc.shift = 0;
    sc.start = pr->ego_speed;
    sc.target = v;
    sc.ttime = fabs(pr->ego_speed - v) / P->relaxed_acc;
    if (pr->has_in) sc_add_limit(&sc, pr->in_ts, pr->in_tt);             /* :1425-1431 */
    if (pr->has_l[L]) sc_add_limit(&sc, pr->l_ts[L], pr->l_tt[L]);       /* :1432-1438 */
    return sc;
}

/* ------------------------------------------------------------------------------------------ */
/* exported oracle API (ctypes)                                                                */
/* ------------------------------------------------------------------------------------------ */
int ppo_map_geometry(const double* wx, const double* wy, int n, double* out) {
    OMap m;
    if (n < 2 || omap_init(&m, wx, wy, n)) return -1;
    for (int i = 0; i < n; i++) {
        double* o = out + (4 + 2 * PP_NUM_LANES) * i;
        o[0] = m.ref[i].x; o[1] = m.ref[i].y; o[2] = m.nx[i]; o[3] = m.ny[i];
        for (int r = 0; r < PP_NUM_LANES; r++) { o[4 + 2 * r] = m.lc[i][r].x; o[5 + 2 * r] = m.lc[i][r].y; }
    }
    omap_free(&m);
    return 0;
}

/* Evaluate scenes [s_begin, s_end) of a host batch; outputs indexed by the global scene id.
 * n_draws = D > 1: every scene is prepared and evaluated D times (draw 0 nominal, draws >= 1 with
 * car noise); cost[s * C + d * Cv + c]; decision = first minimum of the draw-averaged cost (sum in
 * draw order, / D); next_x/next_y = that candidate on the nominal scene. */
int ppo_eval_range(const double* wx, const double* wy, int n_wp, const pp_scene_batch* in,
                   const pp_params* P, pp_result* out, int64_t s_begin, int64_t s_end) {
    if (!in || !P || !out || P->n_points <= PP_PREV_KEEP || P->n_points > PP_MAX_POINTS || P->n_speeds < 1 ||
        P->n_speeds > PP_MAX_SPEEDS || in->car_stride > PP_MAX_CARS || P->n_draws < 0 || P->n_draws > PP_MAX_DRAWS)
        return -1;
    const int D = P->n_draws > 1 ? P->n_draws : 1;
    if (D > 1 && out->paths) return -1;
    OMap m;
    if (n_wp < 2 || omap_init(&m, wx, wy, n_wp)) return -1;
    const int NS = P->n_speeds, Cv = PP_NUM_LANES * NS, C = D * Cv, N = P->n_points;
    double gx[PP_MAX_POINTS], gy[PP_MAX_POINTS];
    double* dcost = (double*)malloc(sizeof(double) * (size_t)C);
    for (int64_t s = s_begin; s < s_end; s++) {
        OPrep pr, pr0;
        uint32_t status = 0;
        for (int d = 0; d < D; d++) {
            prep_scene(&m, P, in, s, d, &pr);
            if (d == 0) pr0 = pr;
            status |= pr.status;
            for (int c = 0; c < Cv; c++) {
                int L = c / NS, k = c % NS;
                double v = cand_speed(P, pr.ego_speed, k);
                OSC sc = make_sc(P, &pr, L, v);
                OStats st;
                int ng = build_traj(&m, P, &pr, L, sc, N, gx, gy, &st);
                int isn;
                double cost = cand_cost(P, &pr, L, v, ng, &st, &isn);
                status |= (st.fallback ? PP_ST_FALLBACK : 0) | (st.trunc ? PP_ST_SPLINE_TRUNC : 0) |
                          (isn ? PP_ST_NAN : 0) | (st.override_hit ? PP_ST_ACC_OVERRIDE : 0) |
                          (st.curv_hit ? PP_ST_CURV_ADJUST : 0);
                dcost[d * Cv + c] = cost;
                if (out->cost) out->cost[s * C + d * Cv + c] = cost;
                if (out->paths) {
                    for (int i = 0; i < N; i++) {
                        double px = NAN, py = NAN;
                        if (i < pr.K) { px = pr.prev[i].x; py = pr.prev[i].y; }
                        else if (i - pr.K < ng) { px = gx[i - pr.K]; py = gy[i - pr.K]; }
                        out->paths[((s * N + i) * C + c) * 2 + 0] = px;
                        out->paths[((s * N + i) * C + c) * 2 + 1] = py;
                    }
                }
                if (out->path_len) out->path_len[s * C + c] = pr.K + ng;
            }
        }
        int best = 0;
        double best_cost = 0;
        for (int c = 0; c < Cv; c++) {
            double sum = dcost[c];
            for (int d = 1; d < D; d++) sum += dcost[d * Cv + c];
            const double mean = sum / D;
            if (D > 1 && out->draw_mean_cost) out->draw_mean_cost[s * Cv + c] = mean;
            if (c == 0 || mean < best_cost) { best = c; best_cost = mean; }
        }
        pr = pr0;
        /* winner path: re-run the winning candidate on the nominal scene */
        {
            int L = best / NS, k = best % NS;
            double v = cand_speed(P, pr.ego_speed, k);
            OSC sc = make_sc(P, &pr, L, v);
            OStats st;
            int ng = build_traj(&m, P, &pr, L, sc, N, gx, gy, &st);
            if (out->winner) out->winner[s] = best;
            if (out->n_out) out->n_out[s] = pr.K + ng;
            if (out->next_x && out->next_y) {
                for (int i = 0; i < N; i++) {
                    double px = 0, py = 0;
                    if (i < pr.K) { px = pr.prev[i].x; py = pr.prev[i].y; }
                    else if (i - pr.K < ng) { px = gx[i - pr.K]; py = gy[i - pr.K]; }
                    out->next_x[(int64_t)i * in->n_scenes + s] = px;
                    out->next_y[(int64_t)i * in->n_scenes + s] = py;
                }
            }
        }
        if (out->status) out->status[s] = status;
        if (out->info) {
            pp_scene_info* I = &out->info[s];
            memset(I, 0, sizeof(*I));
            I->ego_x = pr.ego_x; I->ego_y = pr.ego_y; I->ego_speed = pr.ego_speed; I->ego_acc = pr.ego_acc;
            I->ego_s = pr.ego_s; I->ego_d = pr.ego_d; I->ego_vs = pr.ego_vs; I->ego_vd = pr.ego_vd;
            for (int l = 0; l < PP_NUM_LANES; l++) { I->ref_ratio[l] = pr.fr.ratio[l]; I->lane_score[l] = pr.score[l]; }
            I->ref_wp = pr.fr.ref_wp; I->ego_lane = pr.ego_lane; I->target_lane = pr.T;
            I->lane_open_mask = pr.open_mask; I->n_matched_cars = pr.nmatched; I->in_lane_car = pr.in_id;
        }
    }
    free(dcost);
    omap_free(&m);
    return 0;
}

int ppo_eval(const double* wx, const double* wy, int n_wp, const pp_scene_batch* in,
             const pp_params* P, pp_result* out) {
    return ppo_eval_range(wx, wy, n_wp, in, P, out, 0, in ? in->n_scenes : 0);
}

int ppo_num_lanes(void) { return PP_NUM_LANES; }

/* glibc's own sin/cos/atan2 over arrays (kind 0/1/2), each its own libm call (this file is built
 * with -fno-builtin-sin/-cos, as the reference's -O0 build never fuses them into sincos): the
 * checker for pp_libm_eval (csrc/pp_glibcm.h). */
void ppo_libm_batch(int kind, const double* a, const double* b, double* out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = kind == 0 ? sin(a[i]) : kind == 1 ? cos(a[i]) : atan2(a[i], b[i]);
}

int ppo_struct_sizes(int64_t* out4) {
    out4[0] = sizeof(pp_scene_batch);
    out4[1] = sizeof(pp_params);
    out4[2] = sizeof(pp_result);
    out4[3] = sizeof(pp_scene_info);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Closed-loop rollout (include/pp.h pp_rollout): the simulator shim, restated               */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double *len, *tx, *ty; int n; const OMap* m; } OLanes;   /* [lane * n + i] */

static void olanes_init(OLanes* L, const OMap* m) {
    const int n = m->n;
    L->n = n; L->m = m;
    L->len = (double*)malloc(sizeof(double) * PP_NUM_LANES * n);
    L->tx = (double*)malloc(sizeof(double) * PP_NUM_LANES * n);
    L->ty = (double*)malloc(sizeof(double) * PP_NUM_LANES * n);
    for (int r = 0; r < PP_NUM_LANES; r++)
        for (int i = 0; i < n; i++) {
            const int q = wpi(m, i - 1);
            const double dx = m->lc[i][r].x - m->lc[q][r].x, dy = m->lc[i][r].y - m->lc[q][r].y;
            const double len = sqrt(dx * dx + dy * dy);
            L->len[r * n + i] = len;
            L->tx[r * n + i] = (m->lc[i][r].x - m->lc[q][r].x) / len;
            L->ty[r * n + i] = (m->lc[i][r].y - m->lc[q][r].y) / len;
        }
}

/* advance (seg, t) by dist >= 0 along the lane polyline (segment i ends at waypoint i) */
static void o_lane_advance(const OLanes* L, int lane, int* seg, double* t, double dist) {
    const int n = L->n;
    int i = *seg;
    double tt = *t;
    for (int it = 0; it < 4 * n + 8; it++) {
        const double len = L->len[lane * n + i];
        const double rem = (1.0 - tt) * len;
        if (dist <= rem || it == 4 * n + 7) { tt = tt + dist / len; break; }
        dist -= rem; tt = 0.0; i = (i + 1 == n) ? 0 : i + 1;
    }
    *seg = i;
    *t = tt;
}

static void o_traffic_car(const OLanes* L, int lane, int seg, double t, double off, double v,
                          double* x, double* y, double* vx, double* vy) {
    const int n = L->n;
    const int ip = seg == 0 ? n - 1 : seg - 1;
    const P2 A = L->m->lc[ip][lane], B = L->m->lc[seg][lane];
    const double px = A.x + (B.x - A.x) * t, py = A.y + (B.y - A.y) * t;
    const double ux = L->tx[lane * n + seg], uy = L->ty[lane * n + seg];
    *x = px + uy * off;
    *y = py - ux * off;
    *vx = ux * v;
    *vy = uy * v;
}

/* in: host batch with a car table, updated in place; res: per-frame plan buffers (pp_eval layout) */
int ppo_rollout(const double* wx, const double* wy, int n_wp, pp_scene_batch* in, pp_traffic* tr,
                const pp_params* P, const pp_rollout_cfg* cfg, pp_result* res, pp_rollout_log* log) {
    if (!in || !tr || !P || !cfg || !res || !in->tab_valid || P->n_draws > 1 || P->emit_paths ||
        cfg->consume < 1 || tr->n_cars > in->car_stride)
        return -1;
    OMap m;
    if (n_wp < 2 || omap_init(&m, wx, wy, n_wp)) return -1;
    OLanes L;
    olanes_init(&L, &m);
    const int64_t S = in->n_scenes;
    const int N = P->n_points;
    const double range2 = cfg->sensor_range * cfg->sensor_range;
    double* ex = (double*)in->ego_x;
    double* ey = (double*)in->ego_y;
    double* eyaw = (double*)in->ego_yaw_deg;
    double* espd = (double*)in->ego_speed_mph;
    double* px = (double*)in->prev_x;
    double* py = (double*)in->prev_y;
    for (int f = 0; f < cfg->n_frames; f++) {
        if (ppo_eval_range(wx, wy, n_wp, in, P, res, 0, S)) { free(L.len); free(L.tx); free(L.ty); omap_free(&m); return -1; }
        for (int64_t s = 0; s < S; s++) {
            const int n_out = res->n_out[s];
            const int T = res->winner[s] / P->n_speeds;
            const double x0 = ex[s], y0 = ey[s];
            const int64_t fs = (int64_t)f * S + s;
            if (log) {
                if (log->ego_x) log->ego_x[fs] = x0;
                if (log->ego_y) log->ego_y[fs] = y0;
                if (log->ego_speed_mph) log->ego_speed_mph[fs] = espd[s];
                if (log->target_lane) log->target_lane[fs] = T;
                if (log->winner) log->winner[fs] = res->winner[s];
                if (log->n_out) log->n_out[fs] = n_out;
                if (log->status) log->status[fs] = res->status[s];
                if (log->n_cars) log->n_cars[fs] = in->n_cars[s];
                if (log->plan_x)
                    for (int i = 0; i < N; i++) {
                        log->plan_x[((int64_t)f * N + i) * S + s] = res->next_x[(int64_t)i * S + s];
                        log->plan_y[((int64_t)f * N + i) * S + s] = res->next_y[(int64_t)i * S + s];
                    }
            }
            const int kk = n_out < cfg->consume ? n_out : cfg->consume;
            double nx = x0, ny = y0, qx = x0, qy = y0;
            if (kk >= 1) { nx = res->next_x[(int64_t)(kk - 1) * S + s]; ny = res->next_y[(int64_t)(kk - 1) * S + s]; }
            if (kk >= 2) { qx = res->next_x[(int64_t)(kk - 2) * S + s]; qy = res->next_y[(int64_t)(kk - 2) * S + s]; }
            const double dx = nx - qx, dy = ny - qy;
            const double dist = sqrt(dx * dx + dy * dy);
            ex[s] = nx; ey[s] = ny;
            espd[s] = dist * 50 * 2.237;
            if (dist > 0) eyaw[s] = atan2(dy, dx) * 180.0 / O_PI;
            const int np = n_out - kk;
            for (int i = 0; i < PP_PREV_KEEP; i++) {
                const int ok = i < np;
                px[(int64_t)i * S + s] = ok ? res->next_x[(int64_t)(kk + i) * S + s] : 0.0;
                py[(int64_t)i * S + s] = ok ? res->next_y[(int64_t)(kk + i) * S + s] : 0.0;
            }
            ((int32_t*)in->n_prev)[s] = np;
            ((int32_t*)in->prev_target_lane)[s] = T;
            int nc = 0;
            for (int j = 0; j < tr->n_cars; j++) {
                const int64_t tx = (int64_t)j * S + s;
                const int lane = tr->lane[tx];
                int seg = tr->seg[tx];
                double t = tr->t[tx];
                const double v = tr->speed[tx];
                o_lane_advance(&L, lane, &seg, &t, v * 0.02 * cfg->consume);
                tr->seg[tx] = seg; tr->t[tx] = t;
                double cx, cy, cvx, cvy;
                o_traffic_car(&L, lane, seg, t, tr->offset[tx], v, &cx, &cy, &cvx, &cvy);
                const double rx = cx - nx, ry = cy - ny;
                if (rx * rx + ry * ry <= range2 && nc < in->car_stride) {
                    const int64_t ix = (int64_t)nc * S + s;
                    ((int32_t*)in->car_id)[ix] = j;
                    ((double*)in->car_x)[ix] = cx; ((double*)in->car_y)[ix] = cy;
                    ((double*)in->car_vx)[ix] = cvx; ((double*)in->car_vy)[ix] = cvy;
                    nc++;
                }
            }
            ((int32_t*)in->n_cars)[s] = nc;
        }
    }
    free(L.len); free(L.tx); free(L.ty);
    omap_free(&m);
    return 0;
}


// ---- oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY -------------------------------------
// Appended (by oracle/Makefile) after the reference's src/main.cpp:22-1154, so the classes used
// below are the reference's own. This restates the compute body of the onMessage lambda
// (src/main.cpp:1233-1448) for one telemetry frame per scene, with a fresh sensor_fusion_cars map
// per scene, and additionally runs every (lane, speed) candidate through the same classes.
#include "include/pp.h"

namespace refh {

struct Cand { double sc_target; int lane; };

static void select_follow(std::map<int, Car>& cars, double delta_t0, double ego_s, double ego_d,
                          double d_target, int& in_id, double& in_s, int& t_id, double& t_s) {
    // src/main.cpp:1383-1411 (verbatim logic, target lane parameterised)
    in_id = -1; in_s = 0; t_id = -1; t_s = 0;
    for (auto& p : cars) {
        auto& other = p.second;
        double s0 = other.predicted_s(delta_t0);
        double d0 = other.predicted_d(delta_t0);
        if (s0 > ego_s && fabs(d0 - ego_d) < 3) {
            if (in_id == -1 || in_s > s0) { in_id = other.id; in_s = s0; }
        }
        if (s0 >= ego_s - car_length - safety_distance && fabs(d0 - d_target) < 3) {
            if (t_id == -1 || t_s > s0) { t_id = other.id; t_s = s0; }
        }
    }
    if (t_id == in_id) t_id = -1;
}

static void apply_limits(std::map<int, Car>& cars, SpeedController& sc, int in_id, double in_s,
                         int t_id, double t_s, double ego_s, double ego_speed, double ego_acc) {
    if (in_id != -1) {                                                   // :1425-1431
        LimitSpeed ls;
        auto& fc = cars[in_id];
        ls.calculate(fc, in_s, ego_s, ego_speed, ego_acc, true);
        sc.add_limit_breakpoint(ls.target_speed, ls.target_time);
    }
    if (t_id != -1) {                                                    // :1432-1438
        LimitSpeed ls;
        auto& fc = cars[t_id];
        ls.calculate(fc, t_s, ego_s, ego_speed, ego_acc, false);
        sc.add_limit_breakpoint(ls.target_speed, ls.target_time);
    }
}

}  // namespace refh

// The tunables of src/main.cpp:39-49 are mutable globals in the reference; ref_set_params assigns
// them from a pp_params (include/pp.h, same names and meaning) so that non-default parameter sets
// run through the reference's own classes. The horizon (n_points) is settable only in the build
// whose :854/:1039 literals are replaced by ref_n_points (_ref/libppref_n.so, -DPP_REF_NVAR);
// elsewhere any value but 50 is refused (-1). Returns 0.
extern "C" int ref_horizon_variable() {
#ifdef PP_REF_NVAR
    return 1;
#else
    return 0;
#endif
}

extern "C" int ref_set_params(const pp_params* p) {
#ifdef PP_REF_NVAR
    if (p->n_points <= PP_PREV_KEEP || p->n_points > PP_MAX_POINTS) return -1;
#else
    if (p->n_points != 50) return -1;
#endif
    ref_n_points = p->n_points;
    relaxed_acc = p->relaxed_acc;                                        // :39-49
    min_relaxed_acc_while_braking = p->min_relaxed_acc_while_braking;
    maximum_acc = p->maximum_acc;
    max_speed = p->max_speed;
    car_length = p->car_length;
    safety_distance = p->safety_distance;
    keep_distance = p->keep_distance;
    keep_distance_leeway = p->keep_distance_leeway;
    return 0;
}

// Outputs (all host, caller-allocated; N = ref_n_points, 50 unless ref_set_params changed it):
//   ref_next [S][N][2], ref_n [S], ref_T [S]           : the reference frame's own trajectory
//   paths [S][C][N][2] (NaN padded), path_len [S][C]   : every candidate (lane, speed)
//   info [S][8]: ego_s, ego_d, ego_vs, ego_vd, ego_speed, ego_acc, ego_lane, ref_wp
extern "C" int ref_eval(const double* wx, const double* wy, int n_wp, const pp_scene_batch* in,
                        int n_speeds, const double* speed_offsets, int with_frame,
                        double* ref_next, int* ref_n,
                        int* ref_T, double* paths, int* path_len, double* info) {
    const int N = ref_n_points;
    Map map;
    vector<double> X(wx, wx + n_wp), Y(wy, wy + n_wp);
    map.Init(X, Y);
    const int64_t S = in->n_scenes;
    const int C = NUM_LANES * n_speeds;
    for (int64_t s = 0; s < S; s++) {
        double ego_x = in->ego_x[s];
        double ego_y = in->ego_y[s];
        double ego_yaw = in->ego_yaw_deg[s];
        double ego_speed = in->ego_speed_mph[s];
        ego_speed /= 2.237;
        double ego_acc = 0;
        vector<Point> prev_trajectory;
        double delta_t0 = 0;
        Point ego_speed_vector;
        int prev_trajectory_length = 10;
        if (in->n_prev[s] >= prev_trajectory_length) {                   // :1261-1282
            for (int i = 0; i < prev_trajectory_length; i++)
                prev_trajectory.push_back(Point(in->prev_x[i * S + s], in->prev_y[i * S + s]));
            double v2 = (prev_trajectory[prev_trajectory_length - 2] - prev_trajectory[prev_trajectory_length - 3]).length();
            ego_speed_vector = prev_trajectory[prev_trajectory_length - 1] - prev_trajectory[prev_trajectory_length - 2];
            double v3 = ego_speed_vector.length();
            ego_acc = (v3 - v2) * 50;
            ego_speed = v3 * 50;
            ego_speed_vector.x *= 50;
            ego_speed_vector.y *= 50;
            ego_x = prev_trajectory[prev_trajectory_length - 1].x;
            ego_y = prev_trajectory[prev_trajectory_length - 1].y;
            delta_t0 = prev_trajectory_length / 50.0;
        } else if (jump_to_waypoint) {
            Point p = map.get_waypoint(jump_to_waypoint).lane_center[1];
            ego_x = p.x;
            ego_y = p.y;
        }
        map.init_reference_waypoint(ego_x, ego_y);                       // :1299
        int ego_lane;
        double ego_s, ego_d;
        if (!map.lane_matching(ego_x, ego_y, ego_s, ego_d, ego_lane)) {
            ego_s = ego_d = 0;
            ego_lane = 0;
        }
        double ego_vs, ego_vd;
        map.project_speed(ego_speed_vector, map.reference_waypoint_id, &ego_vs, &ego_vd);
        if (ego_acc > maximum_acc) ego_acc = maximum_acc;
        if (ego_acc < -maximum_acc) ego_acc = -maximum_acc;
        std::map<int, Car> sensor_fusion_cars;                           // :1325-1350
        int ncar = in->n_cars[s] < in->car_stride ? in->n_cars[s] : in->car_stride;
        for (int j = 0; j < ncar; j++) {
            int id = in->car_id[j * S + s];
            auto& car = sensor_fusion_cars[id];
            car.id = id;
            car.x = in->car_x[j * S + s];
            car.y = in->car_y[j * S + s];
            car.vx = in->car_vx[j * S + s];
            car.vy = in->car_vy[j * S + s];
            int next_wp_id = 0;
            if (!map.lane_matching(car.x, car.y, car.s, car.d, car.lane, &next_wp_id))
                sensor_fusion_cars.erase(sensor_fusion_cars.find(id));
            else
                map.project_speed(Point(car.vx, car.vy), next_wp_id, &car.vs, &car.vd);
        }
        int target_lane = in->prev_target_lane[s];
        LaneChangePlanner lane_change_planner;                           // :1352-1356
        target_lane = lane_change_planner.calculate_target_lane(sensor_fusion_cars, ego_lane,
                                                                target_lane, ego_s, ego_vs, delta_t0);
        if (target_lane != ego_lane) {                                   // :1358-1369
            double d_of_target_lane = map.get_lane_center_offset(target_lane);
            double predict_t = 1.0;
            double lane_d_diff = fabs(ego_vd * predict_t + ego_d - d_of_target_lane);
            if (lane_d_diff > 6.0) target_lane = ego_lane;
        }
        // the reference frame's own trajectory (:1383-1457)
        if (with_frame) {
            int in_id, t_id;
            double in_s, t_s;
            refh::select_follow(sensor_fusion_cars, delta_t0, ego_s, ego_d,
                                map.get_lane_center_offset(target_lane), in_id, in_s, t_id, t_s);
            SpeedController speed_controller(ego_speed);
            refh::apply_limits(sensor_fusion_cars, speed_controller, in_id, in_s, t_id, t_s, ego_s,
                               ego_speed, ego_acc);
            TrajectoryBuilder trajectory;
            vector<Point> r = trajectory.build(prev_trajectory, ego_x, ego_y, ego_yaw, ego_lane,
                                               target_lane, ego_d, ego_vd, map, speed_controller);
            ref_n[s] = (int)r.size();
            ref_T[s] = target_lane;
            for (int i = 0; i < N; i++) {
                ref_next[(s * N + i) * 2 + 0] = i < (int)r.size() ? r[i].x : 0.0;
                ref_next[(s * N + i) * 2 + 1] = i < (int)r.size() ? r[i].y : 0.0;
            }
        }
        // every candidate (lane L, speed k): SpeedController with target v (k = 0: max_speed)
        for (int c = 0; c < C; c++) {
            int L = c / n_speeds, k = c % n_speeds;
            double v = max_speed;
            if (k > 0) {
                v = ego_speed + speed_offsets[k - 1];
                if (v < 0) v = 0;
                if (v > max_speed) v = max_speed;
            }
            int in_id, t_id;
            double in_s, t_s;
            refh::select_follow(sensor_fusion_cars, delta_t0, ego_s, ego_d,
                                map.get_lane_center_offset(L), in_id, in_s, t_id, t_s);
            SpeedController sc(ego_speed);
            sc.target_speed = v;
            sc.target_time = fabs(ego_speed - v) / relaxed_acc;
            refh::apply_limits(sensor_fusion_cars, sc, in_id, in_s, t_id, t_s, ego_s, ego_speed, ego_acc);
            TrajectoryBuilder tb;
            vector<Point> r = tb.build(prev_trajectory, ego_x, ego_y, ego_yaw, ego_lane, L, ego_d,
                                       ego_vd, map, sc);
            path_len[s * C + c] = (int)r.size();
            for (int i = 0; i < N; i++) {
                double px = i < (int)r.size() ? r[i].x : NAN;
                double py = i < (int)r.size() ? r[i].y : NAN;
                paths[((s * C + c) * N + i) * 2 + 0] = px;
                paths[((s * C + c) * N + i) * 2 + 1] = py;
            }
        }
        double* I = info + s * 8;
        I[0] = ego_s; I[1] = ego_d; I[2] = ego_vs; I[3] = ego_vd; I[4] = ego_speed; I[5] = ego_acc;
        I[6] = ego_lane; I[7] = map.reference_waypoint_id;
    }
    return 0;
}

// ---- closed-loop rollout (include/pp.h pp_rollout semantics) --------------------------------
// The reference frame (src/main.cpp:1233-1457) with the lambda's cross-frame state kept per
// scene exactly as main() keeps it: the std::map<int, Car> sensor_fusion_cars (:1194, stale
// entries included) and target_lane (:1195). The simulator shim around it is ours (restated
// from include/pp.h: drive `consume` points, lane-following traffic, sensor range).
namespace refh {

static void rollout_frame(Map& map, std::map<int, Car>& sensor_fusion_cars, const pp_scene_batch* in,
                          int64_t s, int& target_lane, vector<Point>& out) {
    const int64_t S = in->n_scenes;
    double ego_x = in->ego_x[s];
    double ego_y = in->ego_y[s];
    double ego_yaw = in->ego_yaw_deg[s];
    double ego_speed = in->ego_speed_mph[s];
    ego_speed /= 2.237;
    double ego_acc = 0;
    vector<Point> prev_trajectory;
    double delta_t0 = 0;
    Point ego_speed_vector;
    int prev_trajectory_length = 10;
    if (in->n_prev[s] >= prev_trajectory_length) {                       // :1261-1282
        for (int i = 0; i < prev_trajectory_length; i++)
            prev_trajectory.push_back(Point(in->prev_x[i * S + s], in->prev_y[i * S + s]));
        double v2 = (prev_trajectory[prev_trajectory_length - 2] - prev_trajectory[prev_trajectory_length - 3]).length();
        ego_speed_vector = prev_trajectory[prev_trajectory_length - 1] - prev_trajectory[prev_trajectory_length - 2];
        double v3 = ego_speed_vector.length();
        ego_acc = (v3 - v2) * 50;
        ego_speed = v3 * 50;
        ego_speed_vector.x *= 50;
        ego_speed_vector.y *= 50;
        ego_x = prev_trajectory[prev_trajectory_length - 1].x;
        ego_y = prev_trajectory[prev_trajectory_length - 1].y;
        delta_t0 = prev_trajectory_length / 50.0;
    }
    map.init_reference_waypoint(ego_x, ego_y);                           // :1299
    int ego_lane;
    double ego_s, ego_d;
    if (!map.lane_matching(ego_x, ego_y, ego_s, ego_d, ego_lane)) {
        ego_s = ego_d = 0;
        ego_lane = 0;
    }
    double ego_vs, ego_vd;
    map.project_speed(ego_speed_vector, map.reference_waypoint_id, &ego_vs, &ego_vd);
    if (ego_acc > maximum_acc) ego_acc = maximum_acc;
    if (ego_acc < -maximum_acc) ego_acc = -maximum_acc;
    int ncar = in->n_cars[s] < in->car_stride ? in->n_cars[s] : in->car_stride;
    for (int j = 0; j < ncar; j++) {                                     // :1325-1350
        int id = in->car_id[j * S + s];
        auto& car = sensor_fusion_cars[id];
        car.id = id;
        car.x = in->car_x[j * S + s];
        car.y = in->car_y[j * S + s];
        car.vx = in->car_vx[j * S + s];
        car.vy = in->car_vy[j * S + s];
        int next_wp_id = 0;
        if (!map.lane_matching(car.x, car.y, car.s, car.d, car.lane, &next_wp_id))
            sensor_fusion_cars.erase(sensor_fusion_cars.find(id));
        else
            map.project_speed(Point(car.vx, car.vy), next_wp_id, &car.vs, &car.vd);
    }
    LaneChangePlanner lane_change_planner;                               // :1352-1356
    target_lane = lane_change_planner.calculate_target_lane(sensor_fusion_cars, ego_lane, target_lane,
                                                            ego_s, ego_vs, delta_t0);
    if (target_lane != ego_lane) {                                       // :1358-1369
        double d_of_target_lane = map.get_lane_center_offset(target_lane);
        double lane_d_diff = fabs(ego_vd * 1.0 + ego_d - d_of_target_lane);
        if (lane_d_diff > 6.0) target_lane = ego_lane;
    }
    int in_id, t_id;                                                     // :1383-1438
    double in_s, t_s;
    select_follow(sensor_fusion_cars, delta_t0, ego_s, ego_d, map.get_lane_center_offset(target_lane),
                  in_id, in_s, t_id, t_s);
    SpeedController speed_controller(ego_speed);
    apply_limits(sensor_fusion_cars, speed_controller, in_id, in_s, t_id, t_s, ego_s, ego_speed, ego_acc);
    TrajectoryBuilder trajectory;                                        // :1448
    out = trajectory.build(prev_trajectory, ego_x, ego_y, ego_yaw, ego_lane, target_lane, ego_d, ego_vd,
                           map, speed_controller);
}

}  // namespace refh

extern "C" int ref_num_lanes() { return NUM_LANES; }

// in: host telemetry batch (updated in place; its tab_* are not used: the std::map is the table)
extern "C" int ref_rollout(const double* wx, const double* wy, int n_wp, pp_scene_batch* in,
                           pp_traffic* tr, const pp_rollout_cfg* cfg, pp_rollout_log* log) {
    Map map;
    vector<double> X(wx, wx + n_wp), Y(wy, wy + n_wp);
    map.Init(X, Y);
    const int n = (int)map.waypoints.size();
    vector<double> len(NUM_LANES * n), tx(NUM_LANES * n), ty(NUM_LANES * n);
    for (int r = 0; r < NUM_LANES; r++)
        for (int i = 0; i < n; i++) {
            const int q = (i - 1 + n) % n;
            const Point a = map.waypoints[q].lane_center[r], b = map.waypoints[i].lane_center[r];
            const double dx = b.x - a.x, dy = b.y - a.y;
            len[r * n + i] = sqrt(dx * dx + dy * dy);
            tx[r * n + i] = (b.x - a.x) / len[r * n + i];
            ty[r * n + i] = (b.y - a.y) / len[r * n + i];
        }
    const int64_t S = in->n_scenes;
    const int N = 50;
    const double range2 = cfg->sensor_range * cfg->sensor_range;
    vector<std::map<int, Car>> tables(S);
    double* ex = (double*)in->ego_x;
    double* ey = (double*)in->ego_y;
    double* eyaw = (double*)in->ego_yaw_deg;
    double* espd = (double*)in->ego_speed_mph;
    for (int f = 0; f < cfg->n_frames; f++) {
        for (int64_t s = 0; s < S; s++) {
            int target_lane = in->prev_target_lane[s];
            vector<Point> P;
            refh::rollout_frame(map, tables[s], in, s, target_lane, P);
            const int n_out = (int)P.size();
            const int64_t fs = (int64_t)f * S + s;
            if (log->ego_x) log->ego_x[fs] = ex[s];
            if (log->ego_y) log->ego_y[fs] = ey[s];
            if (log->ego_speed_mph) log->ego_speed_mph[fs] = espd[s];
            if (log->target_lane) log->target_lane[fs] = target_lane;
            if (log->n_out) log->n_out[fs] = n_out;
            if (log->n_cars) log->n_cars[fs] = in->n_cars[s];
            if (log->plan_x)
                for (int i = 0; i < N; i++) {
                    log->plan_x[((int64_t)f * N + i) * S + s] = i < n_out ? P[i].x : 0.0;
                    log->plan_y[((int64_t)f * N + i) * S + s] = i < n_out ? P[i].y : 0.0;
                }
            // simulator shim
            const int kk = n_out < cfg->consume ? n_out : cfg->consume;
            double nx = ex[s], ny = ey[s], qx = ex[s], qy = ey[s];
            if (kk >= 1) { nx = P[kk - 1].x; ny = P[kk - 1].y; }
            if (kk >= 2) { qx = P[kk - 2].x; qy = P[kk - 2].y; }
            const double dx = nx - qx, dy = ny - qy;
            const double dist = sqrt(dx * dx + dy * dy);
            ex[s] = nx; ey[s] = ny;
            espd[s] = dist * 50 * 2.237;
            if (dist > 0) eyaw[s] = atan2(dy, dx) * 180.0 / 3.14159265358979323846;
            const int np = n_out - kk;
            for (int i = 0; i < PP_PREV_KEEP; i++) {
                ((double*)in->prev_x)[i * S + s] = i < np ? P[kk + i].x : 0.0;
                ((double*)in->prev_y)[i * S + s] = i < np ? P[kk + i].y : 0.0;
            }
            ((int32_t*)in->n_prev)[s] = np;
            ((int32_t*)in->prev_target_lane)[s] = target_lane;
            int nc = 0;
            for (int j = 0; j < tr->n_cars; j++) {
                const int64_t k = (int64_t)j * S + s;
                const int lane = tr->lane[k];
                int seg = tr->seg[k];
                double t = tr->t[k];
                const double v = tr->speed[k];
                double dd = v * 0.02 * cfg->consume;
                for (int it = 0; it < 4 * n + 8; it++) {
                    const double L = len[lane * n + seg];
                    const double rem = (1.0 - t) * L;
                    if (dd <= rem || it == 4 * n + 7) { t = t + dd / L; break; }
                    dd -= rem; t = 0.0; seg = (seg + 1 == n) ? 0 : seg + 1;
                }
                tr->seg[k] = seg; tr->t[k] = t;
                const int ip = seg == 0 ? n - 1 : seg - 1;
                const Point a = map.waypoints[ip].lane_center[lane], b = map.waypoints[seg].lane_center[lane];
                const double px = a.x + (b.x - a.x) * t, py = a.y + (b.y - a.y) * t;
                const double ux = tx[lane * n + seg], uy = ty[lane * n + seg];
                const double cx = px + uy * tr->offset[k], cy = py - ux * tr->offset[k];
                const double rx = cx - nx, ry = cy - ny;
                if (rx * rx + ry * ry <= range2 && nc < in->car_stride) {
                    const int64_t ix = (int64_t)nc * S + s;
                    ((int32_t*)in->car_id)[ix] = j;
                    ((double*)in->car_x)[ix] = cx; ((double*)in->car_y)[ix] = cy;
                    ((double*)in->car_vx)[ix] = ux * v; ((double*)in->car_vy)[ix] = uy * v;
                    nc++;
                }
            }
            ((int32_t*)in->n_cars)[s] = nc;
        }
    }
    return 0;
}

// ---- one episode, frame by frame (the reference lambda's state across calls) -----------------
// A session holds what main() holds across onMessage calls: the Map (with its mutable frame
// members), the std::map<int, Car> sensor_fusion_cars (:1194) and target_lane (:1195). Each call
// runs one telemetry frame (scene 0 of `in`, any car ids) and returns the frame's next_x/next_y.
struct RefSession {
    Map map;
    std::map<int, Car> cars;
    int target_lane;
};

extern "C" void* ref_session_new(const double* wx, const double* wy, int n_wp, int target_lane) {
    RefSession* h = new RefSession();
    vector<double> X(wx, wx + n_wp), Y(wy, wy + n_wp);
    h->map.Init(X, Y);
    h->target_lane = target_lane;
    return h;
}

extern "C" int ref_session_frame(void* hp, const pp_scene_batch* in, double* next_xy, int* n_out,
                                 int* target_lane, int* n_table) {
    RefSession* h = (RefSession*)hp;
    vector<Point> P;
    refh::rollout_frame(h->map, h->cars, in, 0, h->target_lane, P);
    const int n = (int)P.size() < 50 ? (int)P.size() : 50;
    for (int i = 0; i < n; i++) { next_xy[2 * i] = P[i].x; next_xy[2 * i + 1] = P[i].y; }
    *n_out = n;
    *target_lane = h->target_lane;
    *n_table = (int)h->cars.size();
    return 0;
}

extern "C" void ref_session_free(void* hp) { delete (RefSession*)hp; }

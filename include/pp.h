/*
 * pp.h — C-ABI of the MI355X batched trajectory-candidate evaluator.
 *
 * This header is the drop-in boundary. It replaces the reference's per-frame websocket glue
 * (Fable3/CarND-Path-Planning-Project, src/main.cpp:1214-1474: the uWS `onMessage` lambda that
 * parses telemetry, runs the planner and replies with next_x/next_y) by a batch interface:
 * many scenes in, per-candidate costs + one winning next_x/next_y path per scene out.
 *
 *   reference interface                         replaced by
 *   ------------------------------------------  -----------------------------------------------
 *   main(): CSV load + Map::Init                pp_map_create / pp_map_destroy
 *     (src/main.cpp:1160-1193, 89-131)
 *   onMessage compute body (src/main.cpp:       pp_eval (batched, device-resident SoA buffers)
 *     1229-1457) for ONE telemetry frame        pp_plan_frame (one frame, host buffers — the
 *                                                 literal onMessage replacement, C = 1)
 *   TrajectoryBuilder::build (src/main.cpp:     every candidate (lane, speed) of pp_eval runs this
 *     565-1049)                                   exact algorithm; see DESIGN.md
 *
 * Plain C: no torch or HIP types cross this boundary. Device pointers are `void*`/typed pointers
 * into HIP device memory (hipMalloc, or torch tensors' data_ptr()). Every entry point returns an
 * int32 status (PP_OK = 0, negative on error) and never throws.
 */
#ifndef PP_H
#define PP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- fixed sizes ------------------------------------------------------------------------- */
#ifndef PP_NUM_LANES        /* src/main.cpp:22 NUM_LANES (a build-time constant there too; the */
#define PP_NUM_LANES   3    /* library is built for one value: pp_num_lanes() reports it)      */
#endif
#define PP_PREV_KEEP   10   /* src/main.cpp:1258 prev_trajectory_length                       */
/* sensor_fusion rows per scene and car-table slots (the simulator reports 12; the reference's
 * std::map<int, Car> has no bound, src/main.cpp:1194): 256 for up to three lanes, 64 beyond (the
 * planner's order-dependent minima carry each winner's iteration index in a 64-bit word) */
#if PP_NUM_LANES <= 3
#define PP_MAX_CARS    256
#else
#define PP_MAX_CARS    64
#endif
/* the Monte-Carlo noise counter's car stride (pp_mc_gauss): fixed, so a seed draws the same noise
 * in every build whatever its PP_MAX_CARS (which never exceeds it) */
#define PP_NOISE_CAR_STRIDE 256
#define PP_MAX_SPEEDS  8    /* target speeds per lane                                          */
#define PP_MAX_POINTS  128  /* horizon N upper bound (reference: 50, src/main.cpp:854,1039)   */
#define PP_MAX_KNOTS   16   /* spline knots: 9 prev + 1 + 5 control points (src/main.cpp:744) */
#define PP_MAX_DRAWS   1024 /* Monte-Carlo sensor-noise draws per scene (pp_params.n_draws)   */

/* ---- status codes ------------------------------------------------------------------------ */
#define PP_OK              0
#define PP_ERR_ARG        -1   /* null pointer / out-of-range size                              */
#define PP_ERR_HIP        -2   /* HIP runtime error                                            */
#define PP_ERR_NOMEM      -3
#define PP_ERR_NODEVICE   -4
#define PP_ERR_STATE      -5   /* PP_DBG_POISON: a device buffer was not in its between-calls state */

/* ---- per-scene status flags (pp_result.status) -------------------------------------------- */
#define PP_ST_EGO_UNMATCHED  (1u << 0)  /* src/main.cpp:1302-1307 "can't lane match ego"        */
#define PP_ST_CAR_UNMATCHED  (1u << 1)  /* src/main.cpp:1336-1340 car erased                    */
#define PP_ST_FALLBACK       (1u << 2)  /* some candidate used the fallback integrator :848     */
#define PP_ST_SPLINE_TRUNC   (1u << 3)  /* some candidate truncated non-monotone knots :833     */
#define PP_ST_NAN            (1u << 4)  /* some candidate produced a NaN cost / bounded walk hit */
#define PP_ST_COLLISION      (1u << 5)  /* LimitSpeed negative gap :1075-1079                   */
#define PP_ST_ACC_OVERRIDE   (1u << 6)  /* some candidate hit the accT override :945-971        */
#define PP_ST_CURV_ADJUST    (1u << 7)  /* some candidate hit the curvature adjust :972-1018    */
#define PP_ST_TOO_FAR        (1u << 8)  /* "target lane too far" rule fired :1358-1369          */
#define PP_ST_BRAKE          (1u << 9)  /* a LimitSpeed returned BRAKE :1109                    */
#define PP_ST_MAXBRAKE       (1u << 10) /* a LimitSpeed returned MAXBRAKE :1101                 */
#define PP_ST_ADJUST         (1u << 11) /* a LimitSpeed returned ADJUST :1131                   */
#define PP_ST_KEEP           (1u << 12) /* a LimitSpeed returned KEEP :1146                     */
#define PP_ST_LANE_CLOSED    (1u << 13) /* some lane was closed by the planner :405-444         */
#define PP_ST_JUMP_RULE      (1u << 14) /* two-lane jump replaced by adjacent/ego lane :473-479 */

/* ---- cost modes --------------------------------------------------------------------------- */
/* PP_COST_REFERENCE: the reference's decision (planner lane, max_speed) always wins; the other
 *   candidates are ranked behind it by the comfort term. winner's next_x/next_y == reference.
 * PP_COST_COMFORT: pure comfort/lane-score cost, argmin is data dependent. */
#define PP_COST_REFERENCE 0
#define PP_COST_COMFORT   1

/* ---- scene batch (SoA; all arrays caller owned, device resident for pp_eval) ------------- */
/* Index conventions: per-scene scalars [s]; prev points [i * n_scenes + s] (i < PP_PREV_KEEP);
 * cars [j * n_scenes + s] (j < car_stride). Car ids of one scene must be ascending over j < n_cars
 * (the reference iterates a std::map<int, Car>, src/main.cpp:1194, 377, 1388). */
typedef struct pp_scene_batch {
    int64_t n_scenes;
    int32_t car_stride;            /* number of car columns (<= PP_MAX_CARS)                  */
    int32_t tab_slots;             /* car-table slots per scene (<= PP_MAX_CARS; see tab_*)    */
    const double*  ego_x;          /* telemetry x, src/main.cpp:1233                           */
    const double*  ego_y;          /* telemetry y                                              */
    const double*  ego_yaw_deg;    /* telemetry yaw (degrees)                                  */
    const double*  ego_speed_mph;  /* telemetry speed (mph), /2.237 at src/main.cpp:1239       */
    const double*  prev_x;         /* previous_path_x[0..9]                                    */
    const double*  prev_y;         /* previous_path_y[0..9]                                    */
    const int32_t* n_prev;         /* previous_path size (>=10 => first 10 used, else none)    */
    const int32_t* prev_target_lane; /* the cross-frame `target_lane` capture, src/main.cpp:1195 */
    const int32_t* n_cars;         /* sensor_fusion rows used (<= car_stride)                  */
    const int32_t* car_id;
    const double*  car_x;
    const double*  car_y;
    const double*  car_vx;
    const double*  car_vy;
    /* Optional persistent car table: the reference's cross-frame `std::map<int, Car>
     * sensor_fusion_cars` (src/main.cpp:1194, 1325-1350). NULL tab_valid = a fresh table every
     * frame. Otherwise the scene's table is tab_slots slots [k * n_scenes + s] in std::map order:
     * slot k holds car id tab_id[k] (ascending over k; tab_id NULL: slot k is id k), and every car
     * id of this frame's sensor_fusion rows is one of the slot ids (pp_plan_frame, pp_serve and the
     * rollout lay the table out over the union of the stored ids and the frame's ids; any int
     * ids). Visiting the slots in order, a reported car is re-matched and its slot overwritten, or
     * erased (valid = 0) when matching fails (:1336-1340); an unreported valid slot is the car's
     * stale entry, which the planner still uses; an invalid unreported slot is no car. */
    int32_t* tab_id;
    int32_t* tab_valid;
    int32_t* tab_lane;
    double*  tab_s;
    double*  tab_d;
    double*  tab_vs;
    double*  tab_vd;
    double*  tab_vx;
    double*  tab_vy;
} pp_scene_batch;

/* ---- parameters ---------------------------------------------------------------------------- */
typedef struct pp_params {
    int32_t n_points;      /* horizon N incl. kept previous points (reference 50)            */
    int32_t n_speeds;      /* speeds per lane: k = 0 is max_speed, k >= 1 uses speed_offsets   */
    int32_t cost_mode;     /* PP_COST_REFERENCE | PP_COST_COMFORT                             */
    int32_t emit_paths;    /* 1: write every candidate's path to pp_result.paths              */
    double  speed_offsets[PP_MAX_SPEEDS]; /* v_k = clamp(ego_speed + speed_offsets[k-1], 0, max_speed) */
    /* tunables, src/main.cpp:39-49 (defaults = reference values) */
    double  relaxed_acc;                    /* 5    */
    double  min_relaxed_acc_while_braking;  /* 4    */
    double  maximum_acc;                    /* 8    */
    double  max_speed;                      /* 22.2 */
    double  car_length;                     /* 4.5  */
    double  safety_distance;                /* 2    */
    double  keep_distance;                  /* 10   */
    double  keep_distance_leeway;           /* 0.5  */
    /* Monte-Carlo sensor noise (BASELINE config 4). n_draws = D > 1
     * evaluates every scene D times: draw 0 is the scene as given, draw d >= 1 perturbs every
     * sensor_fusion car j by (sigma_pos g0, sigma_pos g1, sigma_vel g2, sigma_vel g3) added to
     * (x, y, vx, vy), g = pp_mc_gauss(noise_seed, noise_first_scene + s, d, j, q). Candidates per
     * scene become C = D * 3 * n_speeds, c = (d * 3 + lane) * n_speeds + k. The per-scene decision
     * averages each (lane, k) cost over the draws (summed in draw order, then / D) and takes the
     * first minimum; next_x/next_y are the draw-0 (nominal) trajectory of that (lane, k), winner
     * = lane * n_speeds + k. emit_paths must be 0 when D > 1. */
    int32_t n_draws;                        /* 0 or 1: off                                  */
    int32_t _pad_mc;
    uint64_t noise_seed;
    int64_t noise_first_scene;              /* global index of the batch's scene 0 (shards)  */
    double  noise_pos_sigma;                /* 0.5 m                        */
    double  noise_vel_sigma;                /* 0.5 m/s                                       */
} pp_params;

/* ---- optional per-scene diagnostics (the planner's intermediate state) --------------------- */
typedef struct pp_scene_info {
    double  ego_x, ego_y, ego_speed, ego_acc;      /* after the derivation, src/main.cpp:1261-1320 */
    double  ego_s, ego_d, ego_vs, ego_vd;
    double  ref_ratio[PP_NUM_LANES];               /* Map::reference_waypoint_ratio          */
    double  lane_score[PP_NUM_LANES];              /* LaneChangePlanner scores :450-471       */
    int32_t ref_wp;                                /* Map::reference_waypoint_id             */
    int32_t ego_lane;
    int32_t target_lane;                           /* after planner + too-far rule           */
    int32_t lane_open_mask;
    int32_t n_matched_cars;
    int32_t in_lane_car;                           /* follow car id or -1, :1383-1400         */
    int32_t _pad[2];
} pp_scene_info;

/* ---- results (caller owned; device resident for pp_eval) ---------------------------------- */
/* C = PP_NUM_LANES * n_speeds (times n_draws for Monte-Carlo), candidate c = lane * n_speeds + k.
 * next_x/next_y: point-major like the batch's prev_x/prev_y, [i * n_scenes + s] (i < n_points;
 * points i >= n_out[s] are 0); cost: [s * C + c];
 * paths (emit_paths): [((s * n_points + i) * C + c) * 2 + {0:x, 1:y}], path_len: [s * C + c]. */
typedef struct pp_result {
    int32_t*  winner;
    int32_t*  n_out;          /* points written to next_x/next_y for the scene (<= n_points)  */
    double*   next_x;
    double*   next_y;
    double*   cost;
    uint32_t* status;
    double*   paths;          /* optional (emit_paths)                                          */
    int32_t*  path_len;       /* optional (emit_paths)                                          */
    pp_scene_info* info;      /* optional                                                       */
    double*   draw_mean_cost; /* optional (n_draws > 1): [s * 3 * n_speeds + lane * n_speeds + k],
                                 the draw-averaged cost the decision minimises                  */
} pp_result;

/* ---- API ----------------------------------------------------------------------------------- */
typedef struct pp_map pp_map;

void    pp_params_default(pp_params* p);
int32_t pp_num_candidates(const pp_params* p);
int32_t pp_num_lanes(void);           /* PP_NUM_LANES of this build */
int32_t pp_max_cars(void);            /* PP_MAX_CARS of this build */

/* Map::Init (src/main.cpp:89-131) on the host (bit-identical to the reference's); the lane
 * geometry is uploaded lazily per device. n >= 3 waypoints, any size. */
int32_t pp_map_create(const double* wx, const double* wy, int32_t n, pp_map** out);
/* Map::Init on `device` from DEVICE waypoint arrays: the same formulas
 * with the device's atan2/cos (the reference's lane centres within ~1e-12 m instead of bit for
 * bit); tables mirrored to the host. Maps of any size (> 600 waypoints: the planner reads the map
 * from global memory instead of staging it in LDS). Synchronous on hip_stream. */
int32_t pp_map_create_device(const double* d_wx, const double* d_wy, int32_t n, int32_t device, void* hip_stream,
                             pp_map** out);
int32_t pp_map_destroy(pp_map* m);
/* host copy of the derived geometry: per waypoint {ref.x, ref.y, nx, ny, lc0.x, lc0.y, lc1.x,
 * lc1.y, ...} (4 + 2 * PP_NUM_LANES doubles) — the Map::Init known-answer output. */
int32_t pp_map_geometry(const pp_map* m, double* out, int32_t n);

/* Pre-size the per-device workspace (optional; pp_eval grows it on demand, which allocates). */
int32_t pp_reserve(pp_map* m, int32_t device, int64_t max_scenes);

/* Evaluate a batch. All batch/result pointers are device memory on `device`; `hip_stream` is a
 * hipStream_t (NULL = default stream). Asynchronous w.r.t. the host. Thread-safe: every stream
 * has its own device workspace, so calls on different streams may overlap; calls on one stream
 * run in its order. */
int32_t pp_eval(pp_map* m, const pp_scene_batch* in, const pp_params* prm, pp_result* out,
                int32_t device, void* hip_stream);

/* One telemetry frame, host memory in/out: the onMessage replacement (C = 1, reference decision).
 * prev_x/prev_y hold n_prev points (only the first 10 are read when n_prev >= 10); the car arrays
 * hold n_cars rows (<= PP_MAX_CARS) in any order with any int ids (sorted by id internally, the
 * last row of a repeated id wins, as std::map assignment does). The car table persists across
 * calls like the reference's (see pp_plan_reset); PP_ERR_ARG if the table would hold more than
 * PP_MAX_CARS distinct cars. *target_lane is read (cross-frame state) and updated. Writes up to
 * 50 points. Calls on one map and device are serialised. */
int32_t pp_plan_frame(pp_map* m, int32_t device,
                      double ego_x, double ego_y, double ego_yaw_deg, double ego_speed_mph,
                      const double* prev_x, const double* prev_y, int32_t n_prev,
                      const int32_t* car_id, const double* car_x, const double* car_y,
                      const double* car_vx, const double* car_vy, int32_t n_cars,
                      int32_t* target_lane, double* next_x, double* next_y, int32_t* n_out);

/* Deterministic synthetic scenes (Philox4x32-10 keyed by seed, counter = global scene index),
 * generated on `device` into caller-owned device buffers described by `out` (car_stride = 12).
 * first_scene = global index of out's scene 0 (for multi-GPU shards). */
int32_t pp_synth_scenes(pp_map* m, uint64_t seed, int64_t first_scene, pp_scene_batch* out,
                        int32_t device, void* hip_stream);
/* The same generator on the host (identical bits except ego_yaw_deg, which goes through atan2). */
int32_t pp_synth_scenes_host(const pp_map* m, uint64_t seed, int64_t first_scene,
                             pp_scene_batch* out);

/* ---- closed-loop rollout ------------------------------------------- */
/* A simulator shim closes the loop around the planner: per frame, pp_eval plans every scene, then
 * the simulator drives `consume` points of each plan (the ego ends on point consume-1; speed and
 * yaw from the last two driven points; previous_path = the undriven rest), sets the cross-frame
 * target lane (src/main.cpp:1195) to the plan's lane (winner / n_speeds), advances the traffic by
 * consume * 0.02 s and reports the cars within sensor_range (ascending id) as the next frame's
 * sensor_fusion; the others become stale car-table entries (tab_* above, required). */
typedef struct pp_traffic {        /* device SoA [j * n_scenes + s]; car j has id j, table slot j  */
    int32_t  n_cars;               /* cars per scene (<= PP_MAX_CARS)                               */
    int32_t  _pad;
    int32_t* lane;                 /* lane-centre polyline it follows                              */
    int32_t* seg;                  /* segment (ends at waypoint seg) and fraction t on it          */
    double*  t;
    double*  offset;               /* lateral offset from the lane centre (right-hand normal)      */
    double*  speed;                /* m/s along the lane                                           */
} pp_traffic;

typedef struct pp_rollout_cfg {
    int32_t n_frames;
    int32_t consume;               /* points the simulator drives per frame (>= 1)                 */
    double  sensor_range;          /* metres; cars farther from the ego are not reported           */
} pp_rollout_cfg;

/* Optional per-frame records, [f * n_scenes + s] (plans: [(f * n_points + i) * n_scenes + s]);
 * any pointer may be NULL. The ego fields are the telemetry the frame was planned from. */
typedef struct pp_rollout_log {
    double*   ego_x;
    double*   ego_y;
    double*   ego_speed_mph;
    int32_t*  target_lane;        /* after the frame (the plan's lane)                             */
    int32_t*  winner;
    int32_t*  n_out;
    uint32_t* status;
    int32_t*  n_cars;             /* sensor_fusion rows the frame was planned from                 */
    double*   plan_x;
    double*   plan_y;
} pp_rollout_log;

/* Runs cfg->n_frames frames; `telemetry` (with its car table: tab_slots >= traffic n_cars, slot j
 * = car j, tab_id NULL or j), `traffic` and `result` (per-frame plan buffers, pp_eval layout) are
 * device state updated in place, so consecutive calls continue the episode. n_draws must be <= 1
 * and emit_paths 0. */
int32_t pp_rollout(pp_map* m, pp_scene_batch* telemetry, pp_traffic* traffic,
                   const pp_params* prm, const pp_rollout_cfg* cfg, pp_result* result,
                   pp_rollout_log* log, int32_t device, void* hip_stream);

/* Rollout start state: writes the synthetic scenes of pp_synth_scenes (same seed and indices)
 * into `telemetry` and their traffic into `out` (n_cars = 12): car j starts exactly where the
 * scene reports it, on its lane with its lateral offset and speed. Empties the car table of
 * `telemetry` when its tab_valid is set. */
int32_t pp_synth_traffic(pp_map* m, uint64_t seed, int64_t first_scene, pp_scene_batch* telemetry,
                         pp_traffic* out, int32_t device, void* hip_stream);
int32_t pp_synth_traffic_host(const pp_map* m, uint64_t seed, int64_t first_scene,
                              pp_scene_batch* telemetry, pp_traffic* out);

/* A batch in HOST memory (the batched onMessage; what a server calls per tick): stages the
 * scenes — and their car table when tab_valid is set, updated in place — through device memory,
 * runs pp_eval on hip_stream and copies winner, n_out, next_x/next_y, cost and status back into
 * the host pp_result. Synchronous. emit_paths must be 0. */
int32_t pp_plan_batch_host(pp_map* m, int32_t device, pp_scene_batch* host_in, const pp_params* prm,
                           pp_result* host_out, void* hip_stream);

/* pp_plan_frame keeps the reference's car table across calls (per map and device, any ids);
 * pp_plan_reset empties it (a new episode). */
int32_t pp_plan_reset(pp_map* m, int32_t device);

/* ---- simulator wire codec (host code) ----------------------------- */
/* Parses n_msgs socket.io frames `42["telemetry",{...}]` — message m is buf[offsets[m],
 * offsets[m+1]) — into scenes [0, n_msgs) of a HOST batch (out->n_scenes >= n_msgs), exactly as
 * the reference's hasData (helpers.h:15-25) + nlohmann::json parse and field reads
 * (src/main.cpp:1217-1252, 1325-1333) see them: previous_path_x/_y keep their first 10 points and
 * n_prev = their length; sensor_fusion rows in std::map order (ascending id, last row of an id
 * wins). msg_status[m]: 0 telemetry; 1 no data (hasData empty: the reference answers
 * `42["manual",{}]`); 2 telemetry with more distinct cars than car_stride (the first car_stride
 * kept); 3 no "42" prefix or another event (the reference does not answer); -1 malformed (the
 * reference's json::parse or field reads would throw). n_threads host threads (<= 1: the calling
 * thread). */
int32_t pp_telemetry_parse(const char* buf, const int64_t* offsets, int64_t n_msgs, pp_scene_batch* out,
                           int32_t* msg_status, int32_t n_threads);
/* Formats `42["control",{"next_x":[...],"next_y":[...]}]` per scene from HOST next_x/next_y
 * ([i * stride + s], the pp_result layout with stride = n_scenes of the batch) and n_out, as
 * nlohmann::json dump does (%.15g, ".0" for integral values, null for non-finite;
 * src/main.cpp:1461-1464). Message s is out[offsets[s], offsets[s+1]). Returns PP_ERR_NOMEM with
 * offsets[n_scenes] = bytes needed when out_cap is too small. */
int32_t pp_control_format(const double* next_x, const double* next_y, const int32_t* n_out, int64_t n_scenes,
                          int64_t stride, char* out, int64_t out_cap, int64_t* offsets, int32_t n_threads);

/* The same codec on the GPU (one lane per frame; identical parser, number conversions and
 * writer). d_buf: the frames back to back in device memory, 16-byte aligned and readable up to
 * offsets[n] rounded up to 16; d_out: a DEVICE batch (n_scenes >= n_msgs). Statuses as above,
 * plus 4: the frame needs the host codec (a number outside the exact conversions' domain, or more
 * sensor_fusion rows than the batch's car_stride) — its fields are not written. Frames of any
 * number of rows up to car_stride parse on the device. Asynchronous on hip_stream. */
int32_t pp_telemetry_parse_device(const char* d_buf, const int64_t* d_offsets, int64_t n_msgs, pp_scene_batch* d_out,
                                  int32_t* d_status, int32_t device, void* hip_stream);
/* Control messages on the GPU into fixed slots: message s = d_slots[s * slot_bytes, + d_len[s]);
 * d_len[s] = -1 when the host codec must format it (a number outside fmt15g's domain, or the
 * slot too small). slot_bytes a multiple of 16; d_slots 16-byte aligned. Asynchronous. */
int32_t pp_control_format_device(const double* d_next_x, const double* d_next_y, const int32_t* d_n_out,
                                 int64_t n_scenes, int64_t stride, char* d_slots, int64_t slot_bytes,
                                 int32_t* d_len, int32_t device, void* hip_stream);

/* ---- simulator shim (host code) ------------------------------------ */
/* A WebSocket server that speaks what the reference's uWS hub speaks on port 4567
 * (src/main.cpp:1214-1494): text frames with socket.io events; per frame the lambda's answers
 * (telemetry -> `42["control",...]`, a "42" frame without data -> `42["manual",{}]`, anything
 * else -> none). Every tick it takes one pending frame from each connected client and plans all of
 * them in one pp_plan_batch_host call (reference decision, 3 x n_speeds candidates); each
 * connection keeps the lambda's cross-frame state (car table, target_lane = 1 at start). */
typedef struct pp_server_opts {
    const char* host;              /* "127.0.0.1" (NULL: same)                                    */
    int32_t port;                  /* 4567 in the reference; 0 = any free port (see bound_port)    */
    int32_t max_clients;           /* connections served (and batched) at once                     */
    int32_t n_speeds;              /* 1 = the reference's own 3 candidates                         */
    int32_t threads;               /* codec threads                                                */
    int32_t device;
    int32_t _pad;
    int64_t max_frames;            /* return after this many telemetry frames (0: until *stop)     */
} pp_server_opts;

/* Blocking; returns when *stop != 0 (set from another thread) or after max_frames. bound_port
 * receives the listening port once bound; stats (4): telemetry frames, batches, connections
 * accepted, replies sent. */
int32_t pp_serve(pp_map* m, const pp_server_opts* opts, volatile int32_t* stop, int32_t* bound_port,
                 int64_t* stats);
/* RFC 6455 Sec-WebSocket-Accept for a client key (the handshake's known-answer check). */
int32_t pp_ws_accept_key(const char* key, char* out, int32_t cap);

/* Debug switches (process-wide; tests and A/B measurements only). Every key defaults to 0, the
 * library's own choice; results never depend on them (the tests check that bit for bit).
 *   PP_DBG_PREP_GROUP  lanes per evaluation of the scene-preparation kernel K1: 1, 2, 4, 8, 16
 *   PP_DBG_PREP_WAVES  K1's one-lane build: 3 or 4 waves per SIMD
 *   PP_DBG_SHAPE       reference-mode launch shape: PP_SHAPE_SPLIT (k_prep, k_cand, k_emit),
 *                      PP_SHAPE_CAND_SMALL (K1, then K2 + K4 in one launch), PP_SHAPE_STEP (the
 *                      whole step in one launch, small batches)
 *   PP_DBG_POISON      1: every call starts from NaN-filled intermediate buffers (prep workspace,
 *                      winner record, staging copies, new car-table slots) and checks that the
 *                      slow-group bitmap is all zero (PP_ERR_STATE otherwise), so no kernel can pass
 *                      a test on what an earlier call left behind
 *   PP_DBG_SPLIT       multi-stream split of reference-mode batches (2 or 3 parts, each K1 -> K2 ->
 *                      K4 on its own stream; beyond 1,572,864 scenes sequential chunks of ~1,048,576
 *                      scenes, 3 parts each): 1 on for every batch the split can take (reference
 *                      mode without paths or draws, more than 65,536 scenes, at least 2,048), 2 off
 *                      (0: batches of 131,072 scenes and more)
 *   PP_DBG_LAST_PARTS  read-only: the parts the last pp_eval launched, 1 when not split
 *   PP_DBG_SORT_CARS   1: order each scene's cars in a pre-pass (k_sort_cars) so the one-lane K1
 *                      reads them visit-major (coalesced; same results, less fetched, slower),
 *                      2 or 0: K1 sorts and gathers them itself (the default)
 * Returns PP_ERR_ARG for an unknown key or value. */
#define PP_DBG_PREP_GROUP  0
#define PP_DBG_PREP_WAVES  1
#define PP_DBG_SHAPE       2
#define PP_DBG_POISON      3
#define PP_DBG_SPLIT       4
#define PP_DBG_LAST_PARTS  5
#define PP_DBG_SORT_CARS   6
#define PP_DBG_KEYS        7
#define PP_SHAPE_SPLIT      1
#define PP_SHAPE_CAND_SMALL 2
#define PP_SHAPE_STEP       3
int32_t pp_debug_set(int32_t key, int32_t value);
int32_t pp_debug_get(int32_t key);

/* Per-kernel timing with HIP events recorded on the launch stream around every kernel of pp_eval
 * (K1 k_prep, K2 k_cand, K3/K4 k_winner or k_emit; a split call (PP_DBG_SPLIT) times each part on
 * its own stream and counts each stage once, as the span from its earliest part's start to its
 * latest part's end: the parts overlap). enable PP_TIMING_K2 records only K2's two
 * events per launch (an event costs a few microseconds of stream time: the bench's timed region
 * records only what its roofline needs); any other nonzero value, every kernel's. pp_timing_read
 * synchronises on the recorded events, returns the summed milliseconds and launch counts per kernel
 * (k_prep and k_winner/k_emit 0 launches under PP_TIMING_K2), and clears the record. */
#define PP_TIMING_ALL 1
#define PP_TIMING_K2  2
int32_t pp_timing_enable(pp_map* m, int32_t device, int32_t enable);
int32_t pp_timing_read(pp_map* m, int32_t device, double* ms3, int64_t* launches3);

/* The Monte-Carlo noise generator (host copy of the device code; bit-identical): standard-normal-
 * like variate q (0..3 -> x, y, vx, vy) of car j in draw d of global scene `scene`. Irwin-Hall of
 * four 32-bit Philox4x32-10 uniforms (key = seed, counter = {scene, (d*PP_NOISE_CAR_STRIDE + j)*4 + q,
 * 0x4D43}), scaled to unit variance: only exactly rounded arithmetic, no libm. */
double  pp_mc_gauss(uint64_t seed, int64_t scene, int32_t draw, int32_t car, int32_t q);

/* The reference's libm as the kernels compute it (csrc/pp_glibcm.h: glibc 2.35 x86-64 sin, cos,
 * atan2 restated bit for bit; used for the frame's heading and rotations in k_prep, the device
 * Map::Init and the scene generator). Evaluates out[i] = sin(a[i]) (kind 0), cos(a[i]) (kind 1) or
 * atan2(a[i], b[i]) (kind 2) for i < n on `device` (pointers to device memory, on `hip_stream`),
 * or on the host (device = -1, host pointers). sin/cos outside |x| < 105414350 give NaN. For
 * parity tests of the device build against the host libm. */
int32_t pp_libm_eval(int32_t kind, const double* a, const double* b, double* out, int64_t n,
                     int32_t device, void* hip_stream);

/* Library version / build info string. */
const char* pp_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PP_H */

"""ctypes loaders for the parity checkers under oracle/ (TEST INFRASTRUCTURE ONLY).

- ``oracle/liboracle.so``: C restatement of the reference loop (oracle/pp_oracle.c); travels to
  the GPU box.
- ``oracle/_ref/libppref.so``: the reference's own planning classes (src/main.cpp:22-1154,
  helpers.h, spline.h) compiled from /root/reference by oracle/Makefile; used to generate and
  re-check the golden fixtures where the reference exists.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "carnd-path-planning-project_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import ppamd  # noqa: E402  (structures shared with the C-ABI)

# overrides select the builds for another PP_NUM_LANES (tests/test_lanes.py)
ORACLE_SO = os.environ.get("PP_ORACLE_SO") or os.path.join(REPO, "oracle", "liboracle.so")
REF_SO = os.environ.get("PP_REF_SO") or os.path.join(REPO, "oracle", "_ref", "libppref.so")
REF_JSON_SO = os.path.join(REPO, "oracle", "_ref", "libppref_json.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

_dp = C.POINTER(C.c_double)


def load_oracle():
    lib = C.CDLL(ORACLE_SO)
    lib.ppo_eval_range.argtypes = [_dp, _dp, C.c_int, C.POINTER(ppamd.SceneBatch),
                                   C.POINTER(ppamd.Params), C.POINTER(ppamd.Result), C.c_int64,
                                   C.c_int64]
    lib.ppo_eval_range.restype = C.c_int
    lib.ppo_map_geometry.argtypes = [_dp, _dp, C.c_int, _dp]
    lib.ppo_map_geometry.restype = C.c_int
    lib.ppo_struct_sizes.argtypes = [C.POINTER(C.c_int64)]
    lib.ppo_mc_gauss.argtypes = [C.c_uint64, C.c_int64, C.c_int, C.c_int, C.c_int]
    lib.ppo_mc_gauss.restype = C.c_double
    lib.ppo_rollout.argtypes = [_dp, _dp, C.c_int, C.POINTER(ppamd.SceneBatch), C.POINTER(ppamd.Traffic),
                                C.POINTER(ppamd.Params), C.POINTER(ppamd.RolloutCfg), C.POINTER(ppamd.Result),
                                C.POINTER(ppamd.RolloutLog)]
    lib.ppo_rollout.restype = C.c_int
    lib.ppo_num_lanes.restype = C.c_int
    lib.ppo_libm_batch.argtypes = [C.c_int, _dp, _dp, _dp, C.c_int64]
    assert lib.ppo_num_lanes() == ppamd.NUM_LANES, (ORACLE_SO, ppamd.LIB_PATH)
    return lib


def noisy_scenes(olib, scenes, prm, draw, first=0):
    """Materialise draw `draw` of a Monte-Carlo batch on the host: every car's (x, y, vx, vy) plus
    sigma * g (include/pp.h pp_params; same operations and order as the kernels)."""
    out = {k: np.array(v, copy=True) for k, v in scenes.items()}
    if draw == 0:
        return out
    S = out["ego_x"].shape[0]
    J = out["car_x"].shape[0]
    g = np.zeros((4, J, S))
    for s in range(S):
        for j in range(J):
            for q in range(4):
                g[q, j, s] = olib.ppo_mc_gauss(prm.noise_seed, prm.noise_first_scene + first + s, draw, j, q)
    out["car_x"] = out["car_x"] + prm.noise_pos_sigma * g[0]
    out["car_y"] = out["car_y"] + prm.noise_pos_sigma * g[1]
    out["car_vx"] = out["car_vx"] + prm.noise_vel_sigma * g[2]
    out["car_vy"] = out["car_vy"] + prm.noise_vel_sigma * g[3]
    return out


def draw_decision(cost, D, Cv):
    """Per-scene decision of the Monte-Carlo mode: first minimum of the draw-averaged cost (sum in
    draw order, then / D). Returns (mean [S, Cv], winner [S])."""
    c = cost.reshape(cost.shape[0], D, Cv)
    acc = c[:, 0, :].copy()
    for d in range(1, D):
        acc = acc + c[:, d, :]
    mean = acc / D
    return mean, np.argmin(mean, axis=1).astype(np.int32)


def load_ref(path=None):
    path = path or REF_SO
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.ref_set_params.argtypes = [C.POINTER(ppamd.Params)]
    lib.ref_set_params.restype = C.c_int
    lib.ref_horizon_variable.restype = C.c_int
    lib.ref_eval.argtypes = [_dp, _dp, C.c_int, C.POINTER(ppamd.SceneBatch), C.c_int, _dp, C.c_int, _dp,
                             C.POINTER(C.c_int), C.POINTER(C.c_int), _dp, C.POINTER(C.c_int), _dp]
    lib.ref_eval.restype = C.c_int
    lib.ref_rollout.argtypes = [_dp, _dp, C.c_int, C.POINTER(ppamd.SceneBatch), C.POINTER(ppamd.Traffic),
                                C.POINTER(ppamd.RolloutCfg), C.POINTER(ppamd.RolloutLog)]
    lib.ref_rollout.restype = C.c_int
    lib.ref_num_lanes.restype = C.c_int
    assert lib.ref_num_lanes() == ppamd.NUM_LANES, (REF_SO, ppamd.LIB_PATH)
    return lib


def load_ref_session():
    """The reference's own frame code with main()'s cross-frame state (ref_session_*), or None."""
    lib = load_ref()
    if lib is None:
        return None
    lib.ref_session_new.argtypes = [_dp, _dp, C.c_int, C.c_int]
    lib.ref_session_new.restype = C.c_void_p
    lib.ref_session_frame.argtypes = [C.c_void_p, C.POINTER(ppamd.SceneBatch), _dp, C.POINTER(C.c_int),
                                      C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.ref_session_free.argtypes = [C.c_void_p]
    return lib


def _arr(a):
    """float64 ctypes pointer to a (kept alive by the caller's reference to a)."""
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def one_scene(ego, prev, rows, target_lane):
    """A host batch of one telemetry frame (ego x, y, yaw_deg, speed_mph; previous points (n, 2);
    sensor_fusion rows (id, x, y, vx, vy) in the order sent); returns {"struct", arrays...}."""
    J = max(len(rows), 1)
    d = ppamd.alloc_scenes(1, J)
    d["ego_x"][0], d["ego_y"][0], d["ego_yaw_deg"][0], d["ego_speed_mph"][0] = ego
    n = min(len(prev), ppamd.PREV_KEEP)
    d["n_prev"][0] = len(prev)
    d["prev_x"][:n, 0] = [p[0] for p in prev[:n]]
    d["prev_y"][:n, 0] = [p[1] for p in prev[:n]]
    d["prev_target_lane"][0] = target_lane
    d["n_cars"][0] = len(rows)
    for j, (cid, x, y, vx, vy) in enumerate(rows):
        d["car_id"][j, 0] = cid
        d["car_x"][j, 0], d["car_y"][j, 0], d["car_vx"][j, 0], d["car_vy"][j, 0] = x, y, vx, vy
    d["struct"] = ppamd.scene_struct(d)
    return d


def copy_state(scenes, traffic):
    return ({k: np.array(v, copy=True) for k, v in scenes.items()},
            {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in traffic.items()})


def oracle_rollout(lib, wx, wy, scenes, traffic, prm, n_frames, consume=3, sensor_range=300.0,
                   plans=True):
    """C restatement closed loop; scenes/traffic (host, with car table) are updated in place."""
    S = int(scenes["ego_x"].shape[0])
    lg = ppamd.alloc_log(n_frames, S, prm.n_points, plans=plans)
    res = ppamd.alloc_result(S, prm)
    b, T, R, L = (ppamd.scene_struct(scenes), ppamd.traffic_struct(traffic), ppamd.result_struct(res),
                  ppamd.log_struct(lg))
    cfg = ppamd.RolloutCfg(n_frames, consume, float(sensor_range))
    wx = np.ascontiguousarray(wx, np.float64)
    wy = np.ascontiguousarray(wy, np.float64)
    rc = lib.ppo_rollout(wx.ctypes.data_as(_dp), wy.ctypes.data_as(_dp), len(wx), C.byref(b), C.byref(T),
                         C.byref(prm), C.byref(cfg), C.byref(R), C.byref(L))
    assert rc == 0, rc
    return lg


def ref_rollout(lib, wx, wy, scenes, traffic, n_frames, consume=3, sensor_range=300.0, plans=True):
    """The reference's own frame code (persistent std::map car table) in the same closed loop."""
    S = int(scenes["ego_x"].shape[0])
    lg = ppamd.alloc_log(n_frames, S, 50, plans=plans)
    b, T, L = ppamd.scene_struct(scenes), ppamd.traffic_struct(traffic), ppamd.log_struct(lg)
    cfg = ppamd.RolloutCfg(n_frames, consume, float(sensor_range))
    wx = np.ascontiguousarray(wx, np.float64)
    wy = np.ascontiguousarray(wy, np.float64)
    with quiet_stdout():
        rc = lib.ref_rollout(wx.ctypes.data_as(_dp), wy.ctypes.data_as(_dp), len(wx), C.byref(b), C.byref(T),
                             C.byref(cfg), C.byref(L))
    assert rc == 0, rc
    return lg


def highway_map():
    return ppamd.highway_map()


def oracle_eval(lib, wx, wy, scenes, prm, begin=0, end=None, info=True):
    """Run the C restatement on host SoA scenes; returns a numpy result dict."""
    S = int(scenes["ego_x"].shape[0])
    end = S if end is None else end
    r = ppamd.alloc_result(S, prm, info=info)
    if prm.emit_paths:
        r["paths"][:] = np.nan
    b = ppamd.scene_struct(scenes)
    R = ppamd.result_struct(r)
    wx = np.ascontiguousarray(wx, np.float64)
    wy = np.ascontiguousarray(wy, np.float64)
    rc = lib.ppo_eval_range(wx.ctypes.data_as(_dp), wy.ctypes.data_as(_dp), len(wx), C.byref(b),
                            C.byref(prm), C.byref(R), begin, end)
    assert rc == 0, rc
    return r


REF_N_SO = os.path.join(REPO, "oracle", "_ref", "libppref_n.so")


def load_ref_n():
    """The reference built with its two point-count literals (src/main.cpp:854, :1039) replaced by
    a settable horizon (oracle/Makefile _ref/libppref_n.so), or None."""
    lib = load_ref(REF_N_SO)
    if lib is not None:
        assert lib.ref_horizon_variable() == 1
    return lib


def ref_eval(lib, wx, wy, scenes, n_speeds=None, speed_offsets=None, with_frame=True, prm=None):
    """Run the reference-compiled checker. prm (a ppamd.Params) assigns the reference's tunable
    globals (src/main.cpp:39-49) and the horizon (libppref_n.so only; the pristine build refuses
    any N but 50) for this call, and supplies n_speeds/speed_offsets; the defaults are restored
    afterwards."""
    if prm is not None:
        n_speeds = prm.n_speeds
        speed_offsets = [prm.speed_offsets[i] for i in range(n_speeds - 1)]
        assert lib.ref_set_params(C.byref(prm)) == 0, "reference build cannot run these params"
    N = prm.n_points if prm is not None else 50
    S = int(scenes["ego_x"].shape[0])
    Cn = ppamd.NUM_LANES * n_speeds
    out = {"ref_next": np.zeros((S, N, 2)), "ref_n": np.zeros(S, np.int32),
           "ref_T": np.zeros(S, np.int32), "paths": np.full((S, Cn, N, 2), np.nan),
           "path_len": np.zeros((S, Cn), np.int32), "info": np.zeros((S, 8))}
    offs = np.zeros(ppamd.MAX_SPEEDS)
    offs[: len(speed_offsets)] = speed_offsets
    b = ppamd.scene_struct(scenes)
    wx = np.ascontiguousarray(wx, np.float64)
    wy = np.ascontiguousarray(wy, np.float64)
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    dp = lambda a: a.ctypes.data_as(_dp)
    try:
        with quiet_stdout():
            rc = lib.ref_eval(dp(wx), dp(wy), len(wx), C.byref(b), n_speeds, dp(offs), int(with_frame),
                              dp(out["ref_next"]), ip(out["ref_n"]), ip(out["ref_T"]),
                              dp(out["paths"]), ip(out["path_len"]), dp(out["info"]))
    finally:
        if prm is not None:
            dflt = ppamd.default_params()
            assert lib.ref_set_params(C.byref(dflt)) == 0
    assert rc == 0
    return out


class quiet_stdout:
    """The reference prints warnings to stdout ("spline input error", "detected collision"):
    silence fd 1 around a call into it."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        self.devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.devnull, 1)

    def __exit__(self, *a):
        C.CDLL(None).fflush(None)      # drain the reference's printf buffer into /dev/null
        os.dup2(self.saved, 1)
        os.close(self.saved)
        os.close(self.devnull)
        return False


def load_ref_json():
    """The reference's own wire codec (helpers.h hasData + nlohmann json.hpp), or None."""
    if not os.path.exists(REF_JSON_SO):
        return None
    lib = C.CDLL(REF_JSON_SO)
    ip = C.POINTER(C.c_int)
    lib.ref_json_parse.argtypes = [C.c_char_p, _dp, _dp, _dp, C.c_int, ip, ip, _dp, C.c_int, ip]
    lib.ref_json_parse.restype = C.c_int
    lib.ref_json_dump.argtypes = [_dp, _dp, C.c_int, C.c_char_p, C.c_long]
    lib.ref_json_dump.restype = C.c_long
    return lib


def ref_json_parse(lib, msg, cap_cars=64):
    """-> (status, ego[4], prev_x[:10], prev_y[:10], n_prev, ids, cars[n, 4])"""
    ego = np.zeros(4)
    px, py = np.zeros(10), np.zeros(10)
    npv, nc = C.c_int(0), C.c_int(0)
    ids = np.zeros(cap_cars, np.int32)
    cars = np.zeros((cap_cars, 4))
    dp = lambda a: a.ctypes.data_as(_dp)
    with quiet_stdout():
        st = lib.ref_json_parse(msg, dp(ego), dp(px), dp(py), 10, C.byref(npv), ids.ctypes.data_as(C.POINTER(C.c_int)),
                                dp(cars), cap_cars, C.byref(nc))
    n = min(nc.value, cap_cars)
    return st, ego, px, py, npv.value, ids[:n], cars[:n]


def ref_json_dump(lib, x, y):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    cap = 64 + 60 * len(x)
    buf = C.create_string_buffer(cap)
    n = lib.ref_json_dump(x.ctypes.data_as(_dp), y.ctypes.data_as(_dp), len(x), buf, cap)
    assert 0 < n <= cap
    return buf.raw[:n]


# ------------------------------------------------------------------------------------------------
# the parity contract (north_star): HIP result vs the oracle on the same scenes
# ------------------------------------------------------------------------------------------------
TOL = 1e-6        # max |dxy| per point, metres


def max_err(a, b):
    """Largest |a - b| over the finite values. The NaN patterns must be identical, and infinite
    values must be equal on both sides (same sign, same places)."""
    na, nb = np.isnan(a), np.isnan(b)
    assert (na == nb).all(), f"NaN pattern differs at {np.count_nonzero(na != nb)} values"
    ia, ib = np.isinf(a), np.isinf(b)
    assert (ia == ib).all() and (a[ia] == b[ia]).all(), \
        f"infinite values differ at {np.count_nonzero((ia != ib) | (ia & (a != b)))} values"
    fa = ~(na | ia)
    return float(np.abs(a[fa] - b[fa]).max()) if fa.any() else 0.0


def compare(got, ref, check_cost=True):
    """Strict parity of a pp_eval result with the oracle's: winners, output counts, path lengths
    and status words exact; every path point and next_x/next_y within TOL with an identical NaN
    pattern (the reference's standstill 0/0 NaN, src/main.cpp:1025, included: pp_glibcm.h makes
    the frame's trig the reference's libm bit for bit, so both sides take the same branch);
    costs within 1e-9. Returns the largest |dxy|."""
    S, Cn = got["cost"].shape
    e = 0.0
    if "paths" in ref:
        assert (got["path_len"] == ref["path_len"]).all(), \
            f"path_len differs for {int((got['path_len'] != ref['path_len']).sum())} candidates"
        e = max_err(got["paths"], ref["paths"])
        assert e <= TOL, e
    assert (got["winner"] == ref["winner"]).all(), f"winner differs in {int((got['winner'] != ref['winner']).sum())} scenes"
    assert (got["n_out"] == ref["n_out"]).all()
    N = got["next_x"].shape[0]          # next_x/next_y are point-major [N][S]
    live = np.arange(N)[:, None] < got["n_out"][None, :]
    for k in ("next_x", "next_y"):
        ee = max_err(np.where(live, got[k], 0.0), np.where(live, ref[k], 0.0))
        assert ee <= TOL, (k, ee)
        e = max(e, ee)
    if check_cost:
        np.testing.assert_allclose(got["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
    assert (got["status"] == ref["status"].view(np.uint32)).all(), \
        f"status differs in {int((got['status'] != ref['status'].view(np.uint32)).sum())} scenes"
    return e


def glibc_batch(olib, kind, a, b=None):
    """glibc's own sin/cos/atan2 (kind 'sin'/'cos'/'atan2') over float64 arrays, one libm call
    per element (oracle/pp_oracle.c ppo_libm_batch)."""
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b if b is not None else a, np.float64)
    out = np.empty_like(a)
    olib.ppo_libm_batch({"sin": 0, "cos": 1, "atan2": 2}[kind], a.ctypes.data_as(_dp), b.ctypes.data_as(_dp),
                        out.ctypes.data_as(_dp), a.size)
    return out

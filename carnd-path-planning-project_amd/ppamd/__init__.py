"""ppamd — Python bindings (ctypes) over the C-ABI in include/pp.h.

The compute path is the HIP library ``libppamd.so`` built for gfx950 from ``csrc/``; this module
only marshals buffers. Importing it fails loudly if the library is missing: there is no CPU
fallback for the planner (the CPU restatement under ``oracle/`` is test infrastructure only).

Reference interface mirrored: the per-frame ``onMessage`` compute body of
Fable3/CarND-Path-Planning-Project ``src/main.cpp:1229-1457`` (see ``plan_frame``) and, batched,
``TrajectoryBuilder::build`` over a (lane, target speed) candidate grid (see ``evaluate``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PPAMD_LIB") or os.path.join(_HERE, "libppamd.so")   # override: A/B builds


def lib_sha256(path=None):
    """SHA-256 of the loaded HIP library file (bench.py matches profile summaries against it)."""
    import hashlib
    h = hashlib.sha256()
    with open(path or LIB_PATH, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()

def _open():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"ppamd: HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
    # torch (ROCm) bundles its own libamdhip64 (soname libamdhip64.so.7, loaded by path). Load it
    # first so that our DT_NEEDED libamdhip64.so.7 resolves to that same runtime: two HIP runtimes
    # in one process do not share device allocations.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    h = C.CDLL(LIB_PATH)
    h.pp_num_lanes.restype = C.c_int32
    return h


_LIB = _open()
NUM_LANES = int(_LIB.pp_num_lanes())   # PP_NUM_LANES the library was built for (src/main.cpp:22)
PREV_KEEP = 10
_LIB.pp_max_cars.restype = C.c_int32
MAX_CARS = int(_LIB.pp_max_cars())     # PP_MAX_CARS: sensor_fusion rows and car-table slots per scene
MAX_SPEEDS = 8
MAX_POINTS = 128

COST_REFERENCE = 0
COST_COMFORT = 1

STATUS_BITS = {
    "EGO_UNMATCHED": 1 << 0, "CAR_UNMATCHED": 1 << 1, "FALLBACK": 1 << 2, "SPLINE_TRUNC": 1 << 3,
    "NAN": 1 << 4, "COLLISION": 1 << 5, "ACC_OVERRIDE": 1 << 6, "CURV_ADJUST": 1 << 7,
    "TOO_FAR": 1 << 8, "BRAKE": 1 << 9, "MAXBRAKE": 1 << 10, "ADJUST": 1 << 11, "KEEP": 1 << 12,
    "LANE_CLOSED": 1 << 13, "JUMP_RULE": 1 << 14,
}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_up = C.POINTER(C.c_uint32)


class SceneBatch(C.Structure):
    _fields_ = [("n_scenes", C.c_int64), ("car_stride", C.c_int32), ("tab_slots", C.c_int32),
                ("ego_x", C.c_void_p), ("ego_y", C.c_void_p), ("ego_yaw_deg", C.c_void_p),
                ("ego_speed_mph", C.c_void_p), ("prev_x", C.c_void_p), ("prev_y", C.c_void_p),
                ("n_prev", C.c_void_p), ("prev_target_lane", C.c_void_p), ("n_cars", C.c_void_p),
                ("car_id", C.c_void_p), ("car_x", C.c_void_p), ("car_y", C.c_void_p),
                ("car_vx", C.c_void_p), ("car_vy", C.c_void_p),
                ("tab_id", C.c_void_p), ("tab_valid", C.c_void_p), ("tab_lane", C.c_void_p), ("tab_s", C.c_void_p),
                ("tab_d", C.c_void_p), ("tab_vs", C.c_void_p), ("tab_vd", C.c_void_p),
                ("tab_vx", C.c_void_p), ("tab_vy", C.c_void_p)]

TABLE_FIELDS_I = ["tab_id", "tab_valid", "tab_lane"]
TABLE_FIELDS_F = ["tab_s", "tab_d", "tab_vs", "tab_vd", "tab_vx", "tab_vy"]


class Traffic(C.Structure):
    _fields_ = [("n_cars", C.c_int32), ("_pad", C.c_int32), ("lane", C.c_void_p), ("seg", C.c_void_p),
                ("t", C.c_void_p), ("offset", C.c_void_p), ("speed", C.c_void_p)]


class ServerOpts(C.Structure):
    _fields_ = [("host", C.c_char_p), ("port", C.c_int32), ("max_clients", C.c_int32), ("n_speeds", C.c_int32),
                ("threads", C.c_int32), ("device", C.c_int32), ("_pad", C.c_int32), ("max_frames", C.c_int64)]


class RolloutCfg(C.Structure):
    _fields_ = [("n_frames", C.c_int32), ("consume", C.c_int32), ("sensor_range", C.c_double)]


LOG_FIELDS = [("ego_x", "f8"), ("ego_y", "f8"), ("ego_speed_mph", "f8"), ("target_lane", "i4"),
              ("winner", "i4"), ("n_out", "i4"), ("status", "u4"), ("n_cars", "i4")]


class RolloutLog(C.Structure):
    _fields_ = [(k, C.c_void_p) for k, _ in LOG_FIELDS] + [("plan_x", C.c_void_p), ("plan_y", C.c_void_p)]


class Params(C.Structure):
    _fields_ = [("n_points", C.c_int32), ("n_speeds", C.c_int32), ("cost_mode", C.c_int32),
                ("emit_paths", C.c_int32), ("speed_offsets", C.c_double * MAX_SPEEDS),
                ("relaxed_acc", C.c_double), ("min_relaxed_acc_while_braking", C.c_double),
                ("maximum_acc", C.c_double), ("max_speed", C.c_double), ("car_length", C.c_double),
                ("safety_distance", C.c_double), ("keep_distance", C.c_double),
                ("keep_distance_leeway", C.c_double), ("n_draws", C.c_int32), ("_pad_mc", C.c_int32),
                ("noise_seed", C.c_uint64), ("noise_first_scene", C.c_int64),
                ("noise_pos_sigma", C.c_double), ("noise_vel_sigma", C.c_double)]


class SceneInfo(C.Structure):
    _fields_ = [("ego_x", C.c_double), ("ego_y", C.c_double), ("ego_speed", C.c_double),
                ("ego_acc", C.c_double), ("ego_s", C.c_double), ("ego_d", C.c_double),
                ("ego_vs", C.c_double), ("ego_vd", C.c_double), ("ref_ratio", C.c_double * NUM_LANES),
                ("lane_score", C.c_double * NUM_LANES), ("ref_wp", C.c_int32), ("ego_lane", C.c_int32),
                ("target_lane", C.c_int32), ("lane_open_mask", C.c_int32),
                ("n_matched_cars", C.c_int32), ("in_lane_car", C.c_int32), ("_pad", C.c_int32 * 2)]


INFO_DTYPE = np.dtype([("ego_x", "f8"), ("ego_y", "f8"), ("ego_speed", "f8"), ("ego_acc", "f8"),
                       ("ego_s", "f8"), ("ego_d", "f8"), ("ego_vs", "f8"), ("ego_vd", "f8"),
                       ("ref_ratio", "f8", NUM_LANES), ("lane_score", "f8", NUM_LANES), ("ref_wp", "i4"),
                       ("ego_lane", "i4"), ("target_lane", "i4"), ("lane_open_mask", "i4"),
                       ("n_matched_cars", "i4"), ("in_lane_car", "i4"), ("_pad", "i4", 2)])
assert INFO_DTYPE.itemsize == C.sizeof(SceneInfo)


class Result(C.Structure):
    _fields_ = [("winner", C.c_void_p), ("n_out", C.c_void_p), ("next_x", C.c_void_p),
                ("next_y", C.c_void_p), ("cost", C.c_void_p), ("status", C.c_void_p),
                ("paths", C.c_void_p), ("path_len", C.c_void_p), ("info", C.c_void_p),
                ("draw_mean_cost", C.c_void_p)]


# exported symbols of include/pp.h (checked by tests/test_capi.py)
EXPORTS = ["pp_params_default", "pp_num_candidates", "pp_version", "pp_map_create",
           "pp_map_destroy", "pp_map_geometry", "pp_reserve", "pp_eval", "pp_plan_frame",
           "pp_synth_scenes", "pp_synth_scenes_host", "pp_timing_enable", "pp_timing_read",
           "pp_mc_gauss", "pp_rollout", "pp_synth_traffic", "pp_synth_traffic_host", "pp_plan_reset",
           "pp_telemetry_parse", "pp_control_format", "pp_plan_batch_host", "pp_serve", "pp_ws_accept_key",
           "pp_telemetry_parse_device", "pp_control_format_device", "pp_map_create_device",
           "pp_num_lanes", "pp_max_cars", "pp_libm_eval", "pp_debug_set", "pp_debug_get"]


def _load():
    lib = _LIB
    lib.pp_params_default.argtypes = [C.POINTER(Params)]
    lib.pp_params_default.restype = None
    lib.pp_num_candidates.argtypes = [C.POINTER(Params)]
    lib.pp_num_candidates.restype = C.c_int32
    lib.pp_version.restype = C.c_char_p
    lib.pp_map_create.argtypes = [_dp, _dp, C.c_int32, C.POINTER(C.c_void_p)]
    lib.pp_map_create.restype = C.c_int32
    lib.pp_map_create_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                                         C.POINTER(C.c_void_p)]
    lib.pp_map_create_device.restype = C.c_int32
    lib.pp_map_destroy.argtypes = [C.c_void_p]
    lib.pp_map_destroy.restype = C.c_int32
    lib.pp_map_geometry.argtypes = [C.c_void_p, _dp, C.c_int32]
    lib.pp_map_geometry.restype = C.c_int32
    lib.pp_reserve.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
    lib.pp_reserve.restype = C.c_int32
    lib.pp_eval.argtypes = [C.c_void_p, C.POINTER(SceneBatch), C.POINTER(Params),
                            C.POINTER(Result), C.c_int32, C.c_void_p]
    lib.pp_eval.restype = C.c_int32
    lib.pp_synth_scenes.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.POINTER(SceneBatch),
                                    C.c_int32, C.c_void_p]
    lib.pp_synth_scenes.restype = C.c_int32
    lib.pp_synth_scenes_host.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.POINTER(SceneBatch)]
    lib.pp_synth_scenes_host.restype = C.c_int32
    lib.pp_plan_frame.argtypes = [C.c_void_p, C.c_int32, C.c_double, C.c_double, C.c_double,
                                  C.c_double, _dp, _dp, C.c_int32, _ip, _dp, _dp, _dp, _dp,
                                  C.c_int32, _ip, _dp, _dp, _ip]
    lib.pp_plan_frame.restype = C.c_int32
    lib.pp_debug_set.argtypes = [C.c_int32, C.c_int32]
    lib.pp_debug_set.restype = C.c_int32
    lib.pp_debug_get.argtypes = [C.c_int32]
    lib.pp_debug_get.restype = C.c_int32
    lib.pp_timing_enable.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    lib.pp_timing_enable.restype = C.c_int32
    lib.pp_timing_read.argtypes = [C.c_void_p, C.c_int32, _dp, C.POINTER(C.c_int64)]
    lib.pp_timing_read.restype = C.c_int32
    lib.pp_mc_gauss.argtypes = [C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    lib.pp_mc_gauss.restype = C.c_double
    lib.pp_rollout.argtypes = [C.c_void_p, C.POINTER(SceneBatch), C.POINTER(Traffic), C.POINTER(Params),
                               C.POINTER(RolloutCfg), C.POINTER(Result), C.POINTER(RolloutLog), C.c_int32,
                               C.c_void_p]
    lib.pp_rollout.restype = C.c_int32
    lib.pp_synth_traffic.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.POINTER(SceneBatch),
                                     C.POINTER(Traffic), C.c_int32, C.c_void_p]
    lib.pp_synth_traffic.restype = C.c_int32
    lib.pp_synth_traffic_host.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.POINTER(SceneBatch),
                                          C.POINTER(Traffic)]
    lib.pp_synth_traffic_host.restype = C.c_int32
    lib.pp_plan_reset.argtypes = [C.c_void_p, C.c_int32]
    lib.pp_plan_reset.restype = C.c_int32
    lib.pp_telemetry_parse.argtypes = [C.c_char_p, C.POINTER(C.c_int64), C.c_int64, C.POINTER(SceneBatch),
                                       C.POINTER(C.c_int32), C.c_int32]
    lib.pp_telemetry_parse.restype = C.c_int32
    lib.pp_control_format.argtypes = [_dp, _dp, C.POINTER(C.c_int32), C.c_int64, C.c_int64, C.c_char_p,
                                      C.c_int64, C.POINTER(C.c_int64), C.c_int32]
    lib.pp_control_format.restype = C.c_int32
    lib.pp_plan_batch_host.argtypes = [C.c_void_p, C.c_int32, C.POINTER(SceneBatch), C.POINTER(Params),
                                       C.POINTER(Result), C.c_void_p]
    lib.pp_plan_batch_host.restype = C.c_int32
    lib.pp_serve.argtypes = [C.c_void_p, C.POINTER(ServerOpts), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                             C.POINTER(C.c_int64)]
    lib.pp_serve.restype = C.c_int32
    lib.pp_ws_accept_key.argtypes = [C.c_char_p, C.c_char_p, C.c_int32]
    lib.pp_ws_accept_key.restype = C.c_int32
    lib.pp_telemetry_parse_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(SceneBatch), C.c_void_p,
                                              C.c_int32, C.c_void_p]
    lib.pp_telemetry_parse_device.restype = C.c_int32
    lib.pp_control_format_device.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                             C.c_int64, C.c_void_p, C.c_int32, C.c_void_p]
    lib.pp_control_format_device.restype = C.c_int32
    lib.pp_libm_eval.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
    lib.pp_libm_eval.restype = C.c_int32
    return lib


lib = _load()


class PPError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        raise PPError(f"{what} failed with status {rc}")


def default_params(n_speeds=5, n_points=50, cost_mode=COST_REFERENCE, emit_paths=False,
                   speed_offsets=None, n_draws=0, noise_seed=None, noise_first_scene=0) -> Params:
    p = Params()
    lib.pp_params_default(C.byref(p))
    p.n_speeds = n_speeds
    p.n_points = n_points
    p.cost_mode = cost_mode
    p.emit_paths = 1 if emit_paths else 0
    p.n_draws = n_draws
    if noise_seed is not None:
        p.noise_seed = noise_seed
    p.noise_first_scene = noise_first_scene
    if speed_offsets is not None:
        for i, v in enumerate(speed_offsets):
            p.speed_offsets[i] = float(v)
    return p


def _ptr(a):
    """Data pointer of a numpy array or torch tensor (contiguous)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    assert a.is_contiguous()
    return a.data_ptr()


class Map:
    """Map::Init (src/main.cpp:89-131) over waypoint x/y; lane geometry uploaded per device."""

    def __init__(self, wx, wy):
        self.wx = np.ascontiguousarray(wx, dtype=np.float64)
        self.wy = np.ascontiguousarray(wy, dtype=np.float64)
        self.n = len(self.wx)
        h = C.c_void_p()
        _check(lib.pp_map_create(self.wx.ctypes.data_as(_dp), self.wy.ctypes.data_as(_dp),
                                 self.n, C.byref(h)), "pp_map_create")
        self.handle = h

    @classmethod
    def from_device(cls, d_wx, d_wy, device=0, stream=None):
        """pp_map_create_device: Map::Init on the GPU from torch waypoint tensors."""
        self = cls.__new__(cls)
        self.wx = d_wx.detach().cpu().numpy().astype(np.float64)
        self.wy = d_wy.detach().cpu().numpy().astype(np.float64)
        self.n = len(self.wx)
        h = C.c_void_p()
        _check(lib.pp_map_create_device(d_wx.data_ptr(), d_wy.data_ptr(), self.n, device, stream, C.byref(h)),
               "pp_map_create_device")
        self.handle = h
        return self

    def geometry(self) -> np.ndarray:
        out = np.zeros((self.n, 4 + 2 * NUM_LANES), np.float64)
        _check(lib.pp_map_geometry(self.handle, out.ctypes.data_as(_dp), self.n), "pp_map_geometry")
        return out

    def reserve(self, device, max_scenes):
        _check(lib.pp_reserve(self.handle, device, max_scenes), "pp_reserve")

    def timing(self, device, enable=True):
        """Per-kernel HIP-event timing: False off, True every kernel, TIMING_K2 K2's events only."""
        _check(lib.pp_timing_enable(self.handle, device, int(enable)), "pp_timing_enable")

    def read_timing(self, device):
        """(ms per kernel [k_prep, k_cand, k_winner], launches per kernel); clears the record."""
        ms = (C.c_double * 3)()
        n = (C.c_int64 * 3)()
        _check(lib.pp_timing_read(self.handle, device, ms, n), "pp_timing_read")
        return list(ms), list(n)

    def close(self):
        if self.handle:
            lib.pp_map_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


SCENE_FIELDS_F = ["ego_x", "ego_y", "ego_yaw_deg", "ego_speed_mph"]
SCENE_FIELDS_I = ["n_prev", "prev_target_lane", "n_cars"]
CAR_FIELDS_F = ["car_x", "car_y", "car_vx", "car_vy"]


def alloc_scenes(S, car_stride=12, xp="numpy", device=None):
    """SoA scene arrays (numpy on host, or torch on `device`)."""
    if xp == "numpy":
        zf = lambda *sh: np.zeros(sh, np.float64)
        zi = lambda *sh: np.zeros(sh, np.int32)
    else:
        import torch
        zf = lambda *sh: torch.zeros(sh, dtype=torch.float64, device=device)
        zi = lambda *sh: torch.zeros(sh, dtype=torch.int32, device=device)
    d = {k: zf(S) for k in SCENE_FIELDS_F}
    d.update({k: zi(S) for k in SCENE_FIELDS_I})
    d["prev_x"] = zf(PREV_KEEP, S)
    d["prev_y"] = zf(PREV_KEEP, S)
    d["car_id"] = zi(car_stride, S)
    d.update({k: zf(car_stride, S) for k in CAR_FIELDS_F})
    return d


def scene_struct(d) -> SceneBatch:
    b = SceneBatch()
    b.n_scenes = int(d["ego_x"].shape[0])
    b.car_stride = int(d["car_id"].shape[0])
    for k in SCENE_FIELDS_F + SCENE_FIELDS_I + CAR_FIELDS_F + ["prev_x", "prev_y", "car_id"]:
        setattr(b, k, _ptr(d[k]))
    for k in TABLE_FIELDS_I + TABLE_FIELDS_F:
        setattr(b, k, _ptr(d.get(k)))
    if d.get("tab_valid") is not None:
        b.tab_slots = int(d["tab_valid"].shape[0])
    return b


def _mk(xp, device):
    if xp == "numpy":
        return (lambda sh: np.zeros(sh, np.float64)), (lambda sh: np.zeros(sh, np.int32))
    import torch
    return (lambda sh: torch.zeros(sh, dtype=torch.float64, device=device),
            lambda sh: torch.zeros(sh, dtype=torch.int32, device=device))


def add_car_table(d, slots=12, xp="numpy", device=None):
    """Adds the persistent car table (include/pp.h tab_*: `slots` slots per scene, slot j = id j,
    empty) to a scene dict."""
    S = int(d["ego_x"].shape[0])
    zf, zi = _mk(xp, device)
    for k in TABLE_FIELDS_I:
        d[k] = zi((slots, S))
    for k in TABLE_FIELDS_F:
        d[k] = zf((slots, S))
    for j in range(slots):
        d["tab_id"][j] = j
    return d


def alloc_traffic(S, n=12, xp="numpy", device=None):
    zf, zi = _mk(xp, device)
    return {"n_cars": 0, "lane": zi((n, S)), "seg": zi((n, S)), "t": zf((n, S)),
            "offset": zf((n, S)), "speed": zf((n, S))}


def traffic_struct(t) -> Traffic:
    T = Traffic()
    T.n_cars = int(t["n_cars"])
    for k in ["lane", "seg", "t", "offset", "speed"]:
        setattr(T, k, _ptr(t[k]))
    return T


def synth_traffic(m, S, seed=0x5EED0001, first=0, device=0, stream=None, car_stride=12):
    """Rollout start state on the GPU: (scenes with an empty car table, traffic)."""
    import torch
    dev = torch.device("cuda", device)
    d = add_car_table(alloc_scenes(S, car_stride, xp="torch", device=dev), xp="torch", device=dev)
    t = alloc_traffic(S, xp="torch", device=dev)
    b, T = scene_struct(d), traffic_struct(t)
    _check(lib.pp_synth_traffic(m.handle, seed, first, C.byref(b), C.byref(T), device, stream), "pp_synth_traffic")
    t["n_cars"] = T.n_cars
    return d, t


def synth_traffic_host(m, S, seed=0x5EED0001, first=0, car_stride=12, slots=12):
    d = add_car_table(alloc_scenes(S, car_stride), slots=slots)
    t = alloc_traffic(S)
    b, T = scene_struct(d), traffic_struct(t)
    _check(lib.pp_synth_traffic_host(m.handle, seed, first, C.byref(b), C.byref(T)), "pp_synth_traffic_host")
    t["n_cars"] = T.n_cars
    return d, t


def alloc_log(F, S, N=50, xp="numpy", device=None, plans=True):
    if xp == "numpy":
        mk = lambda sh, dt: np.zeros(sh, dt)
    else:
        import torch
        tdt = {"f8": torch.float64, "i4": torch.int32, "u4": torch.int32}
        mk = lambda sh, dt: torch.zeros(sh, dtype=tdt[dt], device=device)
    lg = {k: mk((F, S), dt) for k, dt in LOG_FIELDS}
    if plans:
        lg["plan_x"] = mk((F, N, S), "f8")
        lg["plan_y"] = mk((F, N, S), "f8")
    return lg


def log_struct(lg) -> RolloutLog:
    L = RolloutLog()
    for k, _ in LOG_FIELDS:
        setattr(L, k, _ptr(lg.get(k)))
    L.plan_x, L.plan_y = _ptr(lg.get("plan_x")), _ptr(lg.get("plan_y"))
    return L


def rollout(m, scenes, traffic, prm, result, n_frames, consume=3, sensor_range=300.0, log=None,
            device=0, stream=None):
    """pp_rollout: n_frames closed-loop frames on the GPU; scenes/traffic/result updated in place."""
    b, T, R = scene_struct(scenes), traffic_struct(traffic), result_struct(result)
    cfg = RolloutCfg(n_frames, consume, float(sensor_range))
    L = log_struct(log) if log is not None else None
    _check(lib.pp_rollout(m.handle, C.byref(b), C.byref(T), C.byref(prm), C.byref(cfg), C.byref(R),
                          C.byref(L) if L is not None else None, device, stream), "pp_rollout")


def plan_reset(m, device=0):
    _check(lib.pp_plan_reset(m.handle, device), "pp_plan_reset")


def scenes_to_numpy(d):
    return {k: (v if isinstance(v, np.ndarray) else v.cpu().numpy()) for k, v in d.items()}


def synth_host(m: Map, S, seed=0x5EED0001, first=0, car_stride=12):
    d = alloc_scenes(S, car_stride)
    b = scene_struct(d)
    _check(lib.pp_synth_scenes_host(m.handle, seed, first, C.byref(b)), "pp_synth_scenes_host")
    return d


def synth_device(m: Map, S, seed=0x5EED0001, first=0, device=0, stream=None, car_stride=12):
    import torch
    d = alloc_scenes(S, car_stride, xp="torch", device=torch.device("cuda", device))
    b = scene_struct(d)
    _check(lib.pp_synth_scenes(m.handle, seed, first, C.byref(b), device, stream), "pp_synth_scenes")
    return d


def alloc_result(S, prm: Params, xp="numpy", device=None, info=False):
    D = max(prm.n_draws, 1)
    Cn = D * NUM_LANES * prm.n_speeds
    N = prm.n_points
    if xp == "numpy":
        mk = lambda sh, dt: np.zeros(sh, dt)
        f8, i4, u4 = np.float64, np.int32, np.uint32
    else:
        import torch
        mk = lambda sh, dt: torch.zeros(sh, dtype=dt, device=device)
        f8, i4, u4 = torch.float64, torch.int32, torch.int32
    # next_x/next_y are point-major [N][S] (include/pp.h)
    r = {"winner": mk((S,), i4), "n_out": mk((S,), i4), "next_x": mk((N, S), f8),
         "next_y": mk((N, S), f8), "cost": mk((S, Cn), f8), "status": mk((S,), u4)}
    if prm.emit_paths:
        r["paths"] = mk((S, N, Cn, 2), f8)
        r["path_len"] = mk((S, Cn), i4)
    if D > 1:
        r["draw_mean_cost"] = mk((S, NUM_LANES * prm.n_speeds), f8)
    if info:
        if xp == "numpy":
            r["info"] = np.zeros((S,), INFO_DTYPE)
        else:
            import torch
            r["info"] = torch.zeros((S, INFO_DTYPE.itemsize), dtype=torch.uint8, device=device)
    return r


def result_struct(r) -> Result:
    R = Result()
    for k in ["winner", "n_out", "next_x", "next_y", "cost", "status", "paths", "path_len", "info",
              "draw_mean_cost"]:
        setattr(R, k, _ptr(r.get(k)))
    return R


def result_to_numpy(r):
    out = {}
    for k, v in r.items():
        a = v if isinstance(v, np.ndarray) else v.cpu().numpy()
        if k == "status":
            a = a.view(np.uint32)
        if k == "info" and a.dtype == np.uint8:
            a = a.view(INFO_DTYPE).reshape(-1)
        out[k] = a
    return out


def evaluate(m: Map, scenes, prm: Params, result, device=0, stream=None):
    """pp_eval over device-resident scene/result buffers (torch tensors on cuda:device)."""
    b = scene_struct(scenes)
    R = result_struct(result)
    _check(lib.pp_eval(m.handle, C.byref(b), C.byref(prm), C.byref(R), device, stream), "pp_eval")


def plan_frame(m: Map, ego_x, ego_y, ego_yaw_deg, ego_speed_mph, prev_x, prev_y, cars,
               target_lane=1, device=0):
    """The onMessage replacement (src/main.cpp:1229-1466) for one telemetry frame.

    cars: iterable of (id, x, y, vx, vy[, s, d]) rows, as in the simulator's sensor_fusion.
    Returns (next_x, next_y, new_target_lane).
    """
    px = np.ascontiguousarray(prev_x, np.float64)
    py = np.ascontiguousarray(prev_y, np.float64)
    rows = [tuple(r)[:5] for r in cars]
    ids = np.array([int(r[0]) for r in rows], np.int32)
    cx = np.array([r[1] for r in rows], np.float64)
    cy = np.array([r[2] for r in rows], np.float64)
    cvx = np.array([r[3] for r in rows], np.float64)
    cvy = np.array([r[4] for r in rows], np.float64)
    tl = C.c_int32(target_lane)
    nx = np.zeros(50, np.float64)
    ny = np.zeros(50, np.float64)
    n_out = C.c_int32(0)
    _check(lib.pp_plan_frame(m.handle, device, ego_x, ego_y, ego_yaw_deg, ego_speed_mph,
                             px.ctypes.data_as(_dp), py.ctypes.data_as(_dp), len(px),
                             ids.ctypes.data_as(_ip), cx.ctypes.data_as(_dp),
                             cy.ctypes.data_as(_dp), cvx.ctypes.data_as(_dp),
                             cvy.ctypes.data_as(_dp), len(rows), C.byref(tl),
                             nx.ctypes.data_as(_dp), ny.ctypes.data_as(_dp), C.byref(n_out)),
           "pp_plan_frame")
    n = n_out.value
    return nx[:n].copy(), ny[:n].copy(), tl.value


DATA_DIR = os.path.join(os.path.dirname(_HERE), "data")


# pp_timing_enable modes (include/pp.h PP_TIMING_*)
TIMING_ALL, TIMING_K2 = 1, 2

# pp_debug_set keys and launch shapes (include/pp.h PP_DBG_*, PP_SHAPE_*)
DBG_PREP_GROUP, DBG_PREP_WAVES, DBG_SHAPE, DBG_POISON, DBG_SPLIT, DBG_LAST_PARTS, DBG_SORT_CARS = 0, 1, 2, 3, 4, 5, 6
SPLIT_AUTO, SPLIT_ON, SPLIT_OFF = 0, 1, 2
SHAPE_AUTO, SHAPE_SPLIT, SHAPE_CAND_SMALL, SHAPE_STEP = 0, 1, 2, 3


def debug_set(key, value):
    """Process-wide debug switch of the library (pp_debug_set; 0 = the library's own choice)."""
    _check(lib.pp_debug_set(key, value), "pp_debug_set")


def debug_get(key):
    return lib.pp_debug_get(key)


class debug:
    """Context manager: `with ppamd.debug(ppamd.DBG_SHAPE, ppamd.SHAPE_SPLIT): ...` sets a debug
    switch and restores its previous value on exit."""

    def __init__(self, key, value):
        self.key, self.value = key, value

    def __enter__(self):
        self.prev = debug_get(self.key)
        debug_set(self.key, self.value)
        return self

    def __exit__(self, *exc):
        debug_set(self.key, self.prev)
        return False


def set_prep_group(lanes):
    """K1 lanes per evaluation (1, 2, 4, 8, 16; 0 = automatic): pp_debug_set(PP_DBG_PREP_GROUP)."""
    debug_set(DBG_PREP_GROUP, lanes)


def highway_map():
    """x, y of the reference's data/highway_map.csv (the only columns the path reads,
    src/main.cpp:1181-1193), stored as float64 in data/highway_map.npz."""
    z = np.load(os.path.join(DATA_DIR, "highway_map.npz"))
    return z["x"].copy(), z["y"].copy()


def version() -> str:
    return lib.pp_version().decode()


LIBM_KINDS = {"sin": 0, "cos": 1, "atan2": 2}


def libm_eval(kind, a, b=None, device=None):
    """pp_libm_eval: the kernels' restated glibc sin/cos/atan2 (csrc/pp_glibcm.h) over a float64
    array; numpy arrays run the host build, torch CUDA tensors the device build."""
    k = LIBM_KINDS[kind]
    if device is None:
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b if b is not None else a, np.float64)
        out = np.empty_like(a)
        _check(lib.pp_libm_eval(k, a.ctypes.data, b.ctypes.data, out.ctypes.data, a.size, -1, None), "pp_libm_eval")
        return out
    import torch
    b = b if b is not None else a
    out = torch.empty_like(a)
    st = torch.cuda.current_stream(device).cuda_stream
    _check(lib.pp_libm_eval(k, a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), device, st), "pp_libm_eval")
    return out


# ---- wire codec (include/pp.h pp_telemetry_parse / pp_control_format; host) ----------------------
def pack_messages(msgs):
    """list of bytes -> (contiguous buffer, int64 offsets[n + 1])"""
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return b"".join(msgs), off


def telemetry_parse(msgs, car_stride=MAX_CARS, threads=8):
    """Socket.io telemetry frames -> (host scene dict, per-message status)."""
    buf, off = pack_messages(msgs)
    n = len(msgs)
    d = alloc_scenes(n, car_stride)
    st = np.zeros(n, np.int32)
    b = scene_struct(d)
    _check(lib.pp_telemetry_parse(buf, off.ctypes.data_as(C.POINTER(C.c_int64)), n, C.byref(b),
                                  st.ctypes.data_as(C.POINTER(C.c_int32)), threads), "pp_telemetry_parse")
    return d, st


def control_format(next_x, next_y, n_out, threads=8):
    """Point-major host next_x/next_y [N][S] + n_out -> list of control messages (bytes)."""
    nx = np.ascontiguousarray(next_x, np.float64)
    ny = np.ascontiguousarray(next_y, np.float64)
    no = np.ascontiguousarray(n_out, np.int32)
    S = no.shape[0]
    off = np.zeros(S + 1, np.int64)
    cap = max(1024, S * 2048)
    while True:
        out = C.create_string_buffer(cap)
        rc = lib.pp_control_format(nx.ctypes.data_as(_dp), ny.ctypes.data_as(_dp),
                                   no.ctypes.data_as(C.POINTER(C.c_int32)), S, nx.shape[-1] if nx.ndim > 1 else S,
                                   out, cap, off.ctypes.data_as(C.POINTER(C.c_int64)), threads)
        if rc == -3:
            cap = int(off[-1]) + 1
            continue
        _check(rc, "pp_control_format")
        raw = out.raw
        return [raw[off[i]:off[i + 1]] for i in range(S)]


def plan_batch_host(m, scenes, prm, device=0):
    """pp_plan_batch_host: host scene dict (optionally with a car table, updated in place) ->
    host result dict (winner, n_out, next_x/next_y [N][S], cost, status)."""
    S = int(scenes["ego_x"].shape[0])
    r = alloc_result(S, prm)
    _check(lib.pp_plan_batch_host(m.handle, device, C.byref(scene_struct(scenes)), C.byref(prm),
                                  C.byref(result_struct(r)), None), "pp_plan_batch_host")
    return r


class Server:
    """pp_serve on a background thread (ctypes releases the GIL for the blocking call)."""

    def __init__(self, m, port=0, max_clients=64, n_speeds=1, threads=4, device=0, max_frames=0):
        import threading
        self.m = m
        self.opts = ServerOpts(b"127.0.0.1", port, max_clients, n_speeds, threads, device, 0, max_frames)
        self.stop_flag = C.c_int32(0)
        self.port = C.c_int32(0)
        self.stats = (C.c_int64 * 4)()
        self.rc = None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()
        import time
        t0 = time.time()
        while self.port.value == 0 and self.rc is None and time.time() - t0 < 10:
            time.sleep(0.005)
        if self.port.value == 0:
            raise PPError(f"pp_serve did not start (rc={self.rc})")

    def _run(self):
        self.rc = lib.pp_serve(self.m.handle, C.byref(self.opts), C.byref(self.stop_flag), C.byref(self.port),
                               self.stats)

    def close(self):
        self.stop_flag.value = 1
        self.thread.join(timeout=30)
        return self.rc, list(self.stats)


MSG_HOST = 4                      # device codec: the frame needs the host codec


def upload_messages(msgs, device=0):
    """Frames -> (16-byte aligned padded uint8 device buffer, int64 device offsets)."""
    import torch
    buf, off = pack_messages(msgs)
    n = (len(buf) + 15) // 16 * 16 + 16
    host = np.zeros(n, np.uint8)
    host[:len(buf)] = np.frombuffer(buf, np.uint8)
    dev = torch.device("cuda", device)
    return torch.from_numpy(host).to(dev), torch.from_numpy(off).to(dev)


def telemetry_parse_device(msgs, car_stride=MAX_CARS, device=0, stream=None, d_buf=None, d_off=None):
    """pp_telemetry_parse_device -> (device scene dict, device status)."""
    import torch
    dev = torch.device("cuda", device)
    if d_buf is None:
        d_buf, d_off = upload_messages(msgs, device)
    n = int(d_off.shape[0]) - 1
    d = alloc_scenes(n, car_stride, xp="torch", device=dev)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    b = scene_struct(d)
    _check(lib.pp_telemetry_parse_device(d_buf.data_ptr(), d_off.data_ptr(), n, C.byref(b), st.data_ptr(), device,
                                         stream), "pp_telemetry_parse_device")
    return d, st


def control_format_device(next_x, next_y, n_out, slot_bytes=2560, device=0, stream=None):
    """pp_control_format_device on torch [N][S] tensors -> (slots uint8 [S, slot_bytes], len int32 [S])."""
    import torch
    S = int(n_out.shape[0])
    slots = torch.empty((S, slot_bytes), dtype=torch.uint8, device=next_x.device)
    ln = torch.empty(S, dtype=torch.int32, device=next_x.device)
    _check(lib.pp_control_format_device(next_x.data_ptr(), next_y.data_ptr(), n_out.data_ptr(), S,
                                        int(next_x.shape[-1]), slots.data_ptr(), slot_bytes, ln.data_ptr(), device,
                                        stream), "pp_control_format_device")
    return slots, ln


def slots_to_messages(slots, lens):
    """Host copies of device slots -> list of bytes (None where the host codec must format)."""
    sl = slots if isinstance(slots, np.ndarray) else slots.cpu().numpy()
    ln = lens if isinstance(lens, np.ndarray) else lens.cpu().numpy()
    return [bytes(sl[i, :ln[i]]) if ln[i] >= 0 else None for i in range(len(ln))]

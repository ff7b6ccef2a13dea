"""The C-ABI library loads, exports every symbol include/pp.h declares, its struct layouts agree
with the C compiler's view, and argument validation fails cleanly — no GPU compute here."""
import ctypes as C
import os
import re

import numpy as np

import oracle_lib
from oracle_lib import ppamd

HEADER = os.path.join(oracle_lib.REPO, "include", "pp.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|void|double|const char\*)\s+(pp_\w+)\s*\(", txt, re.M)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 12
    assert sorted(ppamd.EXPORTS) == names
    lib = C.CDLL(ppamd.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n


def test_library_is_gfx950_hip():
    data = open(ppamd.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert "gfx950" in ppamd.version()


def test_struct_layouts_match_c():
    sizes = (C.c_int64 * 4)()
    oracle_lib.load_oracle().ppo_struct_sizes(sizes)
    assert list(sizes) == [C.sizeof(ppamd.SceneBatch), C.sizeof(ppamd.Params),
                           C.sizeof(ppamd.Result), C.sizeof(ppamd.SceneInfo)]


def test_params_default_are_reference_constants():
    p = ppamd.default_params()
    # src/main.cpp:39-49
    assert (p.relaxed_acc, p.min_relaxed_acc_while_braking, p.maximum_acc, p.max_speed) == (5, 4, 8, 22.2)
    assert (p.car_length, p.safety_distance, p.keep_distance, p.keep_distance_leeway) == (4.5, 2, 10, 0.5)
    assert p.n_points == 50 and ppamd.lib.pp_num_candidates(C.byref(p)) == 15


def test_argument_validation_without_gpu():
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params()
    b = ppamd.SceneBatch()
    R = ppamd.Result()
    b.n_scenes = 4
    # null pointers -> PP_ERR_ARG before any HIP call
    assert ppamd.lib.pp_eval(m.handle, C.byref(b), C.byref(prm), C.byref(R), 0, None) == -1
    bad = ppamd.default_params(n_points=10)     # must exceed the 10 kept points
    assert ppamd.lib.pp_eval(m.handle, C.byref(b), C.byref(bad), C.byref(R), 0, None) == -1
    bad = ppamd.default_params(n_speeds=9)
    assert ppamd.lib.pp_eval(m.handle, C.byref(b), C.byref(bad), C.byref(R), 0, None) == -1
    assert ppamd.lib.pp_eval(None, C.byref(b), C.byref(prm), C.byref(R), 0, None) == -1
    assert ppamd.lib.pp_eval(m.handle, C.byref(b), C.byref(prm), C.byref(R), 99, None) == -1
    h = C.c_void_p()
    x = np.zeros(2)
    assert ppamd.lib.pp_map_create(x.ctypes.data_as(ppamd._dp), x.ctypes.data_as(ppamd._dp), 2, C.byref(h)) == -1
    x = np.zeros(5)      # duplicate waypoints: Map::Init would divide by zero
    assert ppamd.lib.pp_map_create(x.ctypes.data_as(ppamd._dp), x.ctypes.data_as(ppamd._dp), 5, C.byref(h)) == -1
    assert ppamd.lib.pp_timing_read(m.handle, 99, None, None) == -1


def test_plan_batch_host_null_inputs_rejected_without_gpu():
    """pp_plan_batch_host gathers small batches into its pinned mirror with host memcpy, so every
    host input pointer it would read is checked first: a NULL field (here: each field once, and
    one table array with the table enabled) is PP_ERR_ARG before any HIP call, never a crash."""
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params()
    S = 4
    sc = ppamd.alloc_scenes(S, 12)
    res = ppamd.alloc_result(S, prm)
    R = ppamd.result_struct(res)
    fields = ["ego_x", "ego_y", "ego_yaw_deg", "ego_speed_mph", "prev_x", "prev_y", "n_prev",
              "prev_target_lane", "n_cars", "car_id", "car_x", "car_y", "car_vx", "car_vy"]
    for f in fields:
        b = ppamd.scene_struct(sc)
        setattr(b, f, None)
        assert ppamd.lib.pp_plan_batch_host(m.handle, 0, C.byref(b), C.byref(prm), C.byref(R), None) == -1, f
    tab = {k: np.zeros((12, S), np.int32 if k in ("tab_valid", "tab_lane") else np.float64)
           for k in ("tab_valid", "tab_lane", "tab_s", "tab_d", "tab_vs", "tab_vd", "tab_vx", "tab_vy")}
    for f in tab:
        if f == "tab_valid":
            continue
        b = ppamd.scene_struct(sc)
        b.tab_slots = 12
        for k, v in tab.items():
            setattr(b, k, v.ctypes.data)
        setattr(b, f, None)
        assert ppamd.lib.pp_plan_batch_host(m.handle, 0, C.byref(b), C.byref(prm), C.byref(R), None) == -1, f

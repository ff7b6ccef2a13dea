"""Where one pp_plan_frame call's time goes (diagnostic build -DPP_FRAME_PROF, tools/variants.sh
fprof "-DPP_FRAME_PROF"): host staging, the launch call, launch-to-done, done-to-return (host
clock) and the frame kernel's input copy, body and output copy (device clock), averaged over the
frames. GPU box: PPAMD_LIB=.../libppamd_var_fprof.so python3 tools/frame_prof.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
import ppamd  # noqa: E402


def main():
    lib = ppamd.lib
    lib.pp_frame_prof_read.argtypes = [C.POINTER(C.c_double)]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    sc = ppamd.synth_host(m, 1, seed=0x5EED0001, first=12345)
    ego = [float(sc[k][0]) for k in ("ego_x", "ego_y", "ego_yaw_deg", "ego_speed_mph")]
    n_prev = int(sc["n_prev"][0])
    px, py = sc["prev_x"][:n_prev, 0].copy(), sc["prev_y"][:n_prev, 0].copy()
    rows = [(int(sc["car_id"][j, 0]), float(sc["car_x"][j, 0]), float(sc["car_y"][j, 0]),
             float(sc["car_vx"][j, 0]), float(sc["car_vy"][j, 0])) for j in range(int(sc["n_cars"][0]))]
    ids = np.array([r[0] for r in rows], np.int32)
    cols = [np.array([r[k] for r in rows], np.float64) for k in range(1, 5)]
    nx, ny = np.zeros(50), np.zeros(50)
    tl, n_out = C.c_int32(1), C.c_int32(0)
    dp, ip = ppamd._dp, ppamd._ip
    args = (m.handle, 0, *ego, px.ctypes.data_as(dp), py.ctypes.data_as(dp), len(px), ids.ctypes.data_as(ip),
            *[c.ctypes.data_as(dp) for c in cols], len(rows), C.byref(tl), nx.ctypes.data_as(dp),
            nx.ctypes.data_as(dp) if False else ny.ctypes.data_as(dp), C.byref(n_out))
    out = (C.c_double * 8)()
    for rep in range(2):
        for _ in range(2000):
            tl.value = 1
            assert lib.pp_plan_frame(*args) == 0
        lib.pp_frame_prof_read(out)
    v = list(out)
    n = v[7]
    keys = ["host_staging_us", "launch_call_us", "launch_to_done_us", "done_to_return_us",
            "dev_input_copy_us", "dev_body_us", "dev_output_copy_us"]
    print(json.dumps({"frames": n, **{k: v[i] / n for i, k in enumerate(keys)}}))


if __name__ == "__main__":
    main()

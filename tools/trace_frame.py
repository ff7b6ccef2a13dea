"""Phase timeline of one pp_plan_frame call's k_step_small (diagnostic builds, -DPP_TRACE):
K1 (the scene's preparation by 16 lanes), phase A (the lane splines), phase B (the 0.02 s walks)
and the winner's replay (K4 in the block), from the 100 MHz constant clock. Run on the GPU box:
  PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_trace.so python tools/trace_frame.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
import ppamd  # noqa: E402

K1_BASE = 3 << 16
MAXB = 1 << 18


def main():
    lib = C.CDLL(ppamd.LIB_PATH)
    lib.pp_trace_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int64]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    sc = ppamd.synth_host(m, 1, seed=0x5EED0001, first=12345)
    ego = [float(sc["ego_x"][0]), float(sc["ego_y"][0]), float(sc["ego_yaw_deg"][0]), float(sc["ego_speed_mph"][0])]
    n_prev = int(sc["n_prev"][0])
    px, py = sc["prev_x"][:n_prev, 0].copy(), sc["prev_y"][:n_prev, 0].copy()
    rows = [(int(sc["car_id"][j, 0]), float(sc["car_x"][j, 0]), float(sc["car_y"][j, 0]),
             float(sc["car_vx"][j, 0]), float(sc["car_vy"][j, 0])) for j in range(int(sc["n_cars"][0]))]
    buf = np.zeros(8 * MAXB, np.uint64)
    res = []
    ppamd.plan_reset(m)
    for i in range(60):
        ppamd.plan_frame(m, ego[0], ego[1], ego[2], ego[3], px, py, rows, target_lane=1)
        if i < 10:
            continue
        assert lib.pp_trace_read(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), buf.size) == 0
        t = buf.reshape(MAXB, 8).astype(np.int64)
        k = t[K1_BASE - 1]            # k_step_small: start, after K1, after K2 + K4, end
        q = t[K1_BASE - 2]            # K1 of the scene (lane 0): start, ego, row search, walks, pass, finish
        g = t[0]                      # cand_group: start, phase A end, phase B end per wave, end, K4 table
        c = t[K1_BASE - 3]            # constant clock and shader clock at start and end
        res.append({"map_stage_us": (q[0] - k[0]) / 100, "k1_ego_us": (q[1] - q[0]) / 100,
                    "k1_row_search_us": (q[2] - q[1]) / 100, "k1_car_walks_us": (q[3] - q[2]) / 100,
                    "k1_planner_pass_us": (q[4] - q[3]) / 100, "k1_finish_us": (q[5] - q[4]) / 100,
                    "k1_us": (k[1] - k[0]) / 100, "k2_entry_us": (g[0] - k[1]) / 100,
                    "phase_a_us": (g[1] - g[0]) / 100, "phase_b_us": (g[2:6].max() - g[1]) / 100,
                    "k4_table_us": (g[7] - g[6]) / 100, "k4_replay_us": (k[2] - g[7]) / 100,
                    "slow_pass_us": (k[3] - k[2]) / 100, "total_us": (k[3] - k[0]) / 100,
                    "wave1_phase_a_done_us": (t[K1_BASE - 4][0] - k[0]) / 100})
    out = {k: float(np.median([r[k] for r in res])) for k in res[0]}
    print(json.dumps({"what": "k_step_small phases of pp_plan_frame (median of 50 frames, 100 MHz clock)", **out}))


if __name__ == "__main__":
    main()

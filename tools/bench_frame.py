"""BASELINE config 1 latency: one telemetry frame through pp_plan_frame (the onMessage replacement:
host buffers in, next_x/next_y and the target lane out, car table kept across calls), timed per
call on the GPU box, next to the reference's own planning code (oracle/_ref session, one host
core) on the same frame. Prints one JSON line. Run: python tools/bench_frame.py [--frames K]."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ppamd  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    a = ap.parse_args()
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    sc = ppamd.synth_host(m, 1, seed=0x5EED0001, first=12345)
    ego = [float(sc["ego_x"][0]), float(sc["ego_y"][0]), float(sc["ego_yaw_deg"][0]), float(sc["ego_speed_mph"][0])]
    n_prev = int(sc["n_prev"][0])
    px, py = sc["prev_x"][:n_prev, 0].copy(), sc["prev_y"][:n_prev, 0].copy()
    rows = [(int(sc["car_id"][j, 0]), float(sc["car_x"][j, 0]), float(sc["car_y"][j, 0]),
             float(sc["car_vx"][j, 0]), float(sc["car_vy"][j, 0])) for j in range(int(sc["n_cars"][0]))]

    def gpu_frame():
        return ppamd.plan_frame(m, ego[0], ego[1], ego[2], ego[3], px, py, rows, target_lane=1)

    # the C call alone, its arguments marshalled once (what a compiled caller pays: INTEGRATION.md)
    ids = np.array([r[0] for r in rows], np.int32)
    cols = [np.array([r[k] for r in rows], np.float64) for k in range(1, 5)]
    nxa, nya = np.zeros(50), np.zeros(50)
    tl, n_out_c = C.c_int32(1), C.c_int32(0)
    dp, ip = ppamd._dp, ppamd._ip
    args = (m.handle, 0, ego[0], ego[1], ego[2], ego[3], px.ctypes.data_as(dp), py.ctypes.data_as(dp), len(px),
            ids.ctypes.data_as(ip), *[c.ctypes.data_as(dp) for c in cols], len(rows), C.byref(tl),
            nxa.ctypes.data_as(dp), nya.ctypes.data_as(dp), C.byref(n_out_c))
    fn = ppamd.lib.pp_plan_frame

    def c_frame():
        tl.value = 1
        if fn(*args) != 0:
            raise RuntimeError("pp_plan_frame failed")

    ppamd.plan_reset(m)
    for _ in range(a.warmup):
        c_frame()
    per_c = []
    for _ in range(a.frames):
        t = time.perf_counter()
        c_frame()
        per_c.append(time.perf_counter() - t)
    c_us = np.array(per_c) * 1e6
    ppamd.plan_reset(m)
    for _ in range(a.warmup):
        gpu_frame()
    per = []
    for _ in range(a.frames):
        t = time.perf_counter()
        nx, ny, tl_py = gpu_frame()
        per.append(time.perf_counter() - t)
    gpu_us = np.array(per) * 1e6
    out = {"metric": "pp_plan_frame latency per telemetry frame (BASELINE config 1, 12 cars)", "unit": "us",
           "gpu_median_us": float(np.median(c_us)), "gpu_p10_us": float(np.percentile(c_us, 10)),
           "gpu_p90_us": float(np.percentile(c_us, 90)),
           "gpu_what": "the pp_plan_frame C call (arguments marshalled once), host buffers in and out",
           "python_wrapper_median_us": float(np.median(gpu_us)),
           "c_call_same_plan": bool(n_out_c.value == len(nx) and (nxa[:len(nx)] == nx).all() and (nya[:len(ny)] == ny).all()),
           "frames": a.frames, "n_out": len(nx)}
    # the reference's planning code on one host core, same frame (one session, car table kept)
    try:
        rlib = oracle_lib.load_ref_session()
    except Exception as ex:        # oracle/_ref not built here
        rlib = None
        out["reference"] = f"unavailable: {ex}"
    if rlib is not None:
        h = rlib.ref_session_new(oracle_lib._arr(wx), oracle_lib._arr(wy), len(wx), 1)
        one = oracle_lib.one_scene(ego, np.stack([px, py], 1), rows, 1)
        nxy = np.zeros(100)
        n_out, tl_ref, ntab = C.c_int(), C.c_int(), C.c_int()
        sys.stdout.flush()
        saved = os.dup(1)
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)        # the reference's printf warnings stay out of the JSON line
        try:
            ref = []
            for i in range(a.warmup + a.frames):
                t = time.perf_counter()
                rlib.ref_session_frame(h, C.byref(one["struct"]), nxy.ctypes.data_as(oracle_lib._dp),
                                       C.byref(n_out), C.byref(tl_ref), C.byref(ntab))
                if i >= a.warmup:
                    ref.append(time.perf_counter() - t)
        finally:
            C.CDLL(None).fflush(None)
            os.dup2(saved, 1)
            os.close(saved)
            os.close(devnull)
            rlib.ref_session_free(h)
        out["reference_cpu_median_us"] = float(np.median(ref) * 1e6)
        out["reference"] = "src/main.cpp planning classes (oracle/_ref), one host core, planning only (no JSON)"
        out["same_plan"] = bool(n_out.value == len(nx) and
                                np.abs(nxy[:2 * n_out.value].reshape(-1, 2) - np.stack([nx, ny], 1)).max() <= 1e-6)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

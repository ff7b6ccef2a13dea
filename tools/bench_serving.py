"""Serving pipeline throughput: simulator telemetry frames -> pp_telemetry_parse (host threads)
-> pp_plan_batch_host (H2D, pp_eval, D2H) -> pp_control_format, per batch size; beside it the
reference's own per-frame path on one host core (oracle/_ref: nlohmann parse, the planner frame,
dump) where it was built, else the restatement's planner only. Prints one JSON line.

    python tools/bench_serving.py [--batches 1,64,4096,65536] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ppamd  # noqa: E402


def frames_from_scenes(sc):
    S = sc["ego_x"].shape[0]
    out = []
    for s in range(S):
        npv = int(sc["n_prev"][s])
        k = min(npv, 10)
        px = ",".join(repr(float(v)) for v in sc["prev_x"][:k, s])
        py = ",".join(repr(float(v)) for v in sc["prev_y"][:k, s])
        rows = ",".join("[%d,%r,%r,%r,%r,0,0]" % (int(sc["car_id"][j, s]), float(sc["car_x"][j, s]),
                                                   float(sc["car_y"][j, s]), float(sc["car_vx"][j, s]),
                                                   float(sc["car_vy"][j, s])) for j in range(int(sc["n_cars"][s])))
        out.append(('42["telemetry",{"x":%r,"y":%r,"yaw":%r,"speed":%r,"s":0,"d":0,"previous_path_x":[%s],'
                    '"previous_path_y":[%s],"end_path_s":0,"end_path_d":0,"sensor_fusion":[%s]}]'
                    % (float(sc["ego_x"][s]), float(sc["ego_y"][s]), float(sc["ego_yaw_deg"][s]),
                       float(sc["ego_speed_mph"][s]), px, py, rows)).encode())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,64,4096,65536")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params(n_speeds=1)
    Smax = max(int(b) for b in a.batches.split(","))
    sc = ppamd.synth_host(m, Smax, seed=0x5EED0003)
    frames = frames_from_scenes(sc)
    res = {"metric": "served telemetry frames/s (parse + plan + format), 1 MI355X", "rows": []}
    for B in [int(b) for b in a.batches.split(",")]:
        msgs = frames[:B]
        ppamd.plan_batch_host(m, ppamd.telemetry_parse(msgs, threads=a.threads)[0], prm)   # warm
        t = {"parse": 0.0, "plan": 0.0, "format": 0.0}
        for _ in range(a.reps):
            t0 = time.perf_counter()
            d, st = ppamd.telemetry_parse(msgs, threads=a.threads)
            t1 = time.perf_counter()
            r = ppamd.plan_batch_host(m, d, prm)
            t2 = time.perf_counter()
            out = ppamd.control_format(r["next_x"], r["next_y"], r["n_out"], threads=a.threads)
            t3 = time.perf_counter()
            t["parse"] += t1 - t0
            t["plan"] += t2 - t1
            t["format"] += t3 - t2
        tot = sum(t.values()) / a.reps
        res["rows"].append({"batch": B, "frames_per_s": B / tot, "us_per_batch": tot * 1e6,
                            "parse_us": t["parse"] / a.reps * 1e6, "plan_us": t["plan"] / a.reps * 1e6,
                            "format_us": t["format"] / a.reps * 1e6, "threads": a.threads,
                            "bytes_in_per_frame": sum(map(len, msgs)) / B,
                            "bytes_out_per_frame": sum(map(len, out)) / B})
    # the reference's per-frame path on one core
    import oracle_lib
    rj, rlib = oracle_lib.load_ref_json(), oracle_lib.load_ref()
    if rj is not None and rlib is not None:
        n = 2000
        t0 = time.perf_counter()
        for s in range(n):
            oracle_lib.ref_json_parse(rj, frames[s % Smax])
        t1 = time.perf_counter()
        one = {k: np.ascontiguousarray(v[..., :n]) for k, v in sc.items()}
        with oracle_lib.quiet_stdout():
            t2 = time.perf_counter()
            rr = oracle_lib.ref_eval(rlib, wx, wy, one, 1, [], with_frame=True)
            t3 = time.perf_counter()
        t4 = time.perf_counter()
        for s in range(n):
            oracle_lib.ref_json_dump(rj, rr["ref_next"][s, :, 0], rr["ref_next"][s, :, 1])
        t5 = time.perf_counter()
        res["cpu_reference"] = {"frames_per_s": n / ((t1 - t0) + (t3 - t2) + (t5 - t4)), "cores": 1,
                                "parse_us": (t1 - t0) / n * 1e6, "plan_us": (t3 - t2) / n * 1e6,
                                "dump_us": (t5 - t4) / n * 1e6, "kind": "reference",
                                "note": "nlohmann parse via ctypes per frame (includes Python call overhead), "
                                        "reference planner frame + 3 candidates, nlohmann dump"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

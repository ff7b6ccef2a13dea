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
    # the same frames through the GPU codec: bytes H2D -> device parse -> pp_eval on the device batch
    # -> device format -> slots D2H (frames the device hands back are re-done by the host codec)
    import torch
    dev = torch.device("cuda", 0)
    res["rows_device_codec"] = []
    for B in [int(b) for b in a.batches.split(",")]:
        msgs = frames[:B]
        buf, off = ppamd.pack_messages(msgs)
        npad = (len(buf) + 15) // 16 * 16 + 16
        hbuf = torch.zeros(npad, dtype=torch.uint8).pin_memory()
        hbuf[:len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8)
        hoff = torch.from_numpy(off).pin_memory()
        dbuf = torch.empty(npad, dtype=torch.uint8, device=dev)
        doff = torch.empty(len(off), dtype=torch.int64, device=dev)
        r = ppamd.alloc_result(B, prm, xp="torch", device=dev)
        slot = 2560
        hslots = torch.empty((B, slot), dtype=torch.uint8).pin_memory()
        hlen = torch.empty(B, dtype=torch.int32).pin_memory()

        def run():
            dbuf.copy_(hbuf, non_blocking=True)
            doff.copy_(hoff, non_blocking=True)
            d, st = ppamd.telemetry_parse_device(None, car_stride=16, d_buf=dbuf, d_off=doff,
                                                 stream=torch.cuda.current_stream(dev).cuda_stream)
            ppamd.evaluate(m, d, prm, r, device=0, stream=torch.cuda.current_stream(dev).cuda_stream)
            slots, ln = ppamd.control_format_device(r["next_x"], r["next_y"], r["n_out"], slot_bytes=slot,
                                                    stream=torch.cuda.current_stream(dev).cuda_stream)
            hslots.copy_(slots, non_blocking=True)
            hlen.copy_(ln, non_blocking=True)
            torch.cuda.synchronize(dev)
            return st
        st = run()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            st = run()
        t1 = time.perf_counter()
        msgs_out = ppamd.slots_to_messages(hslots.numpy(), hlen.numpy())
        n_host = int((st.cpu().numpy() == ppamd.MSG_HOST).sum()) + sum(m_ is None for m_ in msgs_out)
        # spot check: identical bytes to the host codec path
        hd, _ = ppamd.telemetry_parse(msgs[:256], threads=a.threads)
        hr = ppamd.plan_batch_host(m, hd, prm)
        same = ppamd.control_format(hr["next_x"], hr["next_y"], hr["n_out"])
        agree = sum(int(msgs_out[i] == same[i]) for i in range(min(256, B)))
        tot = (t1 - t0) / a.reps
        res["rows_device_codec"].append({"batch": B, "frames_per_s": B / tot, "us_per_batch": tot * 1e6,
                                         "frames_for_host_codec": n_host, "bytes_h2d": npad, "bytes_d2h": B * slot,
                                         "first_256_identical_to_host_path": agree})
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

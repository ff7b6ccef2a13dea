"""Branch-event census of k_cand's step loop (diagnostic builds, -DPP_DIAG).

Build: tools/variants.sh diag "-DPP_DIAG"; run on the GPU box:
  PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_diag.so python tools/diag_events.py
Per event: the fraction of lane-steps where it fired and of wave-steps where any lane fired (the
wave then executes the branch body). One pp_eval over the bench's synthetic batch.
"""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))

NAMES = ["step", "seg_reload", "ramp_div", "wide_turn", "limiter", "override", "curv_adjust",
         "override_cls1", "wide_first_step", "dt_le_0", "limiter_ng0", "limiter_ng1", "limiter_ng2_4",
         "limiter_ng5_9", "limiter_ng10_19", "limiter_ng20_", "match_walk_step", "car_match", "not_dok",
         "adjust_wide", "loop_entry", "seg_back", "winner_out",
         "adjust_narrow", "match_approach_step"]


def main():
    import argparse
    import torch
    import ppamd
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=262144)
    ap.add_argument("--n-speeds", type=int, default=5)
    ap.add_argument("--n-points", type=int, default=50)
    ap.add_argument("--emit-paths", action="store_true")
    a = ap.parse_args()
    S = a.scenes
    lib = C.CDLL(ppamd.LIB_PATH)
    lib.pp_diag_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params(n_speeds=a.n_speeds, n_points=a.n_points, emit_paths=a.emit_paths,
                               speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if a.n_speeds == 8 else None)
    scenes = ppamd.synth_device(m, S, seed=0x5EED0001, device=0)
    res = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
    buf = (C.c_ulonglong * 96)()
    lib.pp_diag_read(buf, 1)
    ppamd.evaluate(m, scenes, prm, res, device=0)
    torch.cuda.synchronize()
    assert lib.pp_diag_read(buf, 1) == 0
    lanes0, waves0 = buf[0], buf[1]
    out = {"scenes": S, "n_speeds": a.n_speeds, "n_points": a.n_points, "emit_paths": a.emit_paths, "lane_steps": lanes0, "wave_steps": waves0,
           "waves": buf[2 * 20 + 1], "lanes": buf[2 * 20],
           "lanes_per_wave_step": lanes0 / max(waves0, 1)}
    for k, n in enumerate(NAMES):
        if not n or k == 0:
            continue
        out[n] = {"lane_frac": buf[2 * k] / max(lanes0, 1), "wave_frac": buf[2 * k + 1] / max(waves0, 1),
                  "lanes": buf[2 * k], "waves": buf[2 * k + 1]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

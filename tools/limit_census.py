"""Limiter census on the GPU (the -DPP_LIMCENSUS build): one pp_eval over a
BASELINE batch, then the census counters (csrc/pp_eval.hip PP_CEN events 26-33) as one JSON line.

At every decision of the acceleration limiter (src/main.cpp:941 `acc + centrifugal_acceleration >
maximum_acc`, and :972 after the speed override) the census build evaluates, from the same state,
both the kernel's operation sequence (the asin series of the unit-step cross product, the
Markstein-corrected ramp division) and the reference's (glibc atan2 of the step, the wrapped
difference of absolute angles, the IEEE division), and counts:
  near_941 / near_972   decisions whose kernel-side left side lies within a relative 1e-12 of
                        maximum_acc (the knife-edge the SURVEY asks to flag)
  near_941_ref          the same for the reference-side left side
  differ_941 / _972     decisions the two operation sequences take differently
  cacc_bits_differ      steps where the two centrifugal accelerations differ in any bit
  speed_bits_differ     steps where the two ramp speeds differ in any bit
  eval_972              second tests evaluated (lanes)
Each counter is in lanes (candidate-steps); `_waves` is the number of wave-steps with any lane.

GPU box:  PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_census.so \\
          python3 tools/limit_census.py --config 5
"""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))

EVENTS = {26: "near_941", 27: "near_941_ref", 28: "differ_941", 29: "eval_972", 30: "near_972",
          31: "differ_972", 32: "cacc_bits_differ", 33: "speed_bits_differ"}
# BASELINE.json configs 2-5: scenes, speeds, points, all paths, draws
CONFIGS = {2: (4096, 5, 50, False, 0), 3: (262144, 8, 100, True, 0), 4: (16384, 1, 50, False, 64),
           5: (2097152, 5, 50, False, 0)}


def census(config, seed=0x5EED0001, comfort=False):
    import torch
    import ppamd
    S, ns, N, paths, draws = CONFIGS[config]
    lib = C.CDLL(ppamd.LIB_PATH)
    if not hasattr(lib, "pp_diag_read"):
        raise SystemExit(f"{ppamd.LIB_PATH} is not a census build (no pp_diag_read)")
    lib.pp_diag_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params(n_speeds=ns, n_points=N, emit_paths=paths, n_draws=draws,
                               cost_mode=ppamd.COST_COMFORT if comfort else ppamd.COST_REFERENCE,
                               speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if ns == 8 else None)
    dev = torch.device("cuda", 0)
    scenes = ppamd.synth_device(m, S, seed=seed, device=0)
    res = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    torch.cuda.synchronize(dev)
    buf = (C.c_ulonglong * 96)()
    assert lib.pp_diag_read(buf, 1) == 0
    ppamd.evaluate(m, scenes, prm, res, device=0)
    torch.cuda.synchronize(dev)
    assert lib.pp_diag_read(buf, 1) == 0
    out = {"config": config, "scenes": S, "candidates": S * 3 * ns * max(draws, 1), "n_points": N,
           "comfort": comfort, "lib": os.path.basename(ppamd.LIB_PATH)}
    for k, name in EVENTS.items():
        out[name] = int(buf[2 * k])
        out[name + "_waves"] = int(buf[2 * k + 1])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=5, choices=sorted(CONFIGS))
    ap.add_argument("--comfort", action="store_true")
    a = ap.parse_args()
    print(json.dumps(census(a.config, comfort=a.comfort)), flush=True)


if __name__ == "__main__":
    main()

"""Generates tests/golden/rollout_golden.npz: closed-loop replays (SURVEY.md §8(c) golden item
(iii), §8(f) row 1) produced by the REFERENCE's own frame code — oracle/_ref/libppref.so, its
src/main.cpp classes with main()'s persistent std::map car table and target_lane — driven by the
simulator shim of include/pp.h (pp_rollout). Two variants: a sensor range of 120 m (cars leave and
re-enter the sensor list, so the table holds stale entries) and an unlimited one.

Stored: the start state (synthetic scenes + traffic, pp_synth_traffic_host), the per-frame log
(telemetry ego x/y/speed, target lane, plan length, reported cars) for every frame, and the full
plans of the first PLAN_FRAMES frames. The C restatement (oracle/pp_oracle.c ppo_rollout) is
asserted bit-identical to the reference on the same run before anything is written.

Run from the repo root (needs oracle/_ref built by `make -C oracle`):
    python tests/golden/make_rollout_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402

SEED = 0x5EED0007
SCENES = 8
FRAMES = 600
CONSUME = 3
PLAN_FRAMES = 30
VARIANTS = {"r120": 120.0, "rinf": 1.0e4}


def main():
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    olib, rlib = oracle_lib.load_oracle(), oracle_lib.load_ref()
    assert rlib is not None, "oracle/_ref/libppref.so not built"
    prm = ppamd.default_params(n_speeds=1)
    out = {"seed": SEED, "frames": FRAMES, "consume": CONSUME, "plan_frames": PLAN_FRAMES}
    for name, rng in VARIANTS.items():
        sc, tr = ppamd.synth_traffic_host(m, SCENES, seed=SEED)
        for k, v in sc.items():
            out[f"{name}_scene_{k}"] = v.copy()
        for k, v in tr.items():
            out[f"{name}_traffic_{k}"] = np.asarray(v).copy()
        out[f"{name}_range"] = rng
        a = oracle_lib.copy_state(sc, tr)
        b = oracle_lib.copy_state(sc, tr)
        lo = oracle_lib.oracle_rollout(olib, wx, wy, *a, prm, FRAMES, CONSUME, rng)
        lr = oracle_lib.ref_rollout(rlib, wx, wy, *b, FRAMES, CONSUME, rng)
        for k in ["ego_x", "ego_y", "ego_speed_mph", "target_lane", "n_out", "n_cars", "plan_x", "plan_y"]:
            assert np.array_equal(lo[k], lr[k]), (name, k)
            keep = lr[k][:PLAN_FRAMES] if k.startswith("plan") else lr[k]
            out[f"{name}_ref_{k}"] = keep
        print(f"{name}: {SCENES} scenes x {FRAMES} frames, reference == restatement; "
              f"lanes {np.bincount(lr['target_lane'].ravel(), minlength=3)}, "
              f"reported cars/frame {lr['n_cars'].min()}..{lr['n_cars'].max()}")
    np.savez_compressed(os.path.join(HERE, "rollout_golden.npz"), **out)


if __name__ == "__main__":
    main()

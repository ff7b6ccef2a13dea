"""Launch shapes one after another on one stream (a class of tests that passed on
device state an earlier call left behind). pp_eval keeps per-stream workspaces (prep record,
winner record, slow-group bitmap and list) across calls, sized by the largest batch so far; every
shape must produce the oracle's results whatever ran before it. The sequence visits every launch
shape twice, each time right after a different shape and with a different batch size and
candidate count, with speed-edge scenes that route groups to the checked k_cand<true> (the bitmap
k_cand<true> must leave clear):
  split      k_prep + k_cand<false> + k_cand<true> + k_emit (reference decision)
  cand_small K1 (grouped) + k_cand_small
  step       k_step_small (the whole step in one launch)
  paths      emit_paths: k_prep + k_cand<.., 2> (every candidate's path)
  comfort    cost argmin: k_cand<.., 0> + k_winner
  draws      Monte-Carlo draws: k_prep per draw + k_cand<.., 0> + k_winner
  rollout    pp_rollout: frames of pp_eval + k_sim with a car table
The suite runs with PP_DBG_POISON on (tests/conftest.py): intermediates and outputs start
NaN-filled and the bitmap must be clear at every call's entry."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def scenes(env, S, seed):
    sc = ppamd.synth_host(env["m"], S, seed=seed, first=seed * 1000)
    speeds = [-0.0, 5e-324, 1e-300, 3e6, 1e300, -3.0]
    idx = np.arange(3, S, 53)
    sc["n_prev"][idx] = 0
    sc["ego_speed_mph"][idx] = np.array(speeds)[np.arange(len(idx)) % len(speeds)]
    return sc


def run_eval(env, shape, S, seed):
    t = env["torch"]
    sc = scenes(env, S, seed)
    kw = {"split": {}, "cand_small": {}, "step": {}, "paths": {"emit_paths": True, "n_speeds": 8,
                                                               "speed_offsets": [-6, -4, -3, -2, -1, 0, 2]},
          "comfort": {"cost_mode": ppamd.COST_COMFORT, "n_speeds": 3, "speed_offsets": [-3.0, 1.0]},
          "draws": {"n_speeds": 1, "n_draws": 6, "noise_seed": 11}}[shape]
    prm = ppamd.default_params(**kw)
    dbg = {"split": ppamd.SHAPE_SPLIT, "cand_small": ppamd.SHAPE_CAND_SMALL, "step": ppamd.SHAPE_STEP}.get(shape, 0)
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    with ppamd.debug(ppamd.DBG_SHAPE, dbg):
        ppamd.evaluate(env["m"], d, prm, r, device=0)
    t.cuda.synchronize()
    got = ppamd.result_to_numpy(r)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
    return oracle_lib.compare(got, ref)


def run_rollout(env, S, seed):
    t = env["torch"]
    sc, tr = ppamd.synth_traffic_host(env["m"], S, seed=seed)
    a = oracle_lib.copy_state(sc, tr)
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    g = {k: (t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) if isinstance(v, np.ndarray) else v)
         for k, v in tr.items()}
    prm = ppamd.default_params(n_speeds=1)
    F = 12
    res = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    lg = ppamd.alloc_log(F, S, 50, xp="torch", device=env["dev"])
    ppamd.rollout(env["m"], d, g, prm, res, F, 3, 150.0, lg)
    t.cuda.synchronize()
    got = {k: x.cpu().numpy() for k, x in lg.items()}
    lo = oracle_lib.oracle_rollout(env["olib"], env["wx"], env["wy"], *a, prm, F, 3, 150.0)
    for k in ("target_lane", "n_out", "n_cars", "winner", "status"):
        if k in lo and k in got:
            np.testing.assert_array_equal(got[k], lo[k], err_msg=k)
    e = 0.0
    for k in ("ego_x", "ego_y", "plan_x", "plan_y"):
        fin = np.isfinite(lo[k])
        assert (np.isfinite(got[k]) == fin).all(), k
        e = max(e, float(np.abs(got[k][fin] - lo[k][fin]).max()))
    assert e <= oracle_lib.TOL, e
    return e


# every shape twice, each after a different one; sizes and candidate counts change between calls
# (batches grow and shrink, so workspaces are both reused oversized and regrown)
SEQUENCE = [("split", 3000), ("step", 700), ("paths", 1200), ("cand_small", 2500), ("comfort", 900),
            ("draws", 400), ("rollout", 300), ("split", 1500), ("cand_small", 800), ("draws", 900),
            ("paths", 500), ("step", 2000), ("rollout", 128), ("comfort", 2600), ("split", 2200)]


def test_shapes_after_other_shapes(env):
    worst = 0.0
    for i, (shape, S) in enumerate(SEQUENCE):
        seed = 101 + i
        e = run_rollout(env, S, seed) if shape == "rollout" else run_eval(env, shape, S, seed)
        worst = max(worst, e)
        print(f"{i:2d} {shape:10s} S={S:5d} max |dxy| {e:.3e} m")
    assert worst <= oracle_lib.TOL

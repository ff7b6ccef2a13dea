"""The multi-stream split (pp_eval, include/pp.h PP_DBG_SPLIT): reference-mode batches of about a
2-, 4- or 8-GPU shard's size run as 2 parts (up to 393,216 scenes) or 3 parts, each K1 -> K2 -> K4 on
its own stream; larger batches, when the split is forced, as sequential chunks of about 1,048,576
scenes, 3 parts each (round 6). The parts write disjoint ranges of every buffer and keep separate flagged-group
lists, so the results must be the one-stream launch's BIT FOR BIT, including the scenes routed to
k_cand<true> and part boundaries that split no group; a sample is checked against the oracle."""
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


def run(env, sc, prm, mode, group=0):
    t = env["torch"]
    S = sc["ego_x"].shape[0]
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    # (a forced K1 group of 1 also forces the three-kernel shape: small batches run one fused launch)
    shape = ppamd.SHAPE_SPLIT if group == 1 else ppamd.SHAPE_AUTO
    with ppamd.debug(ppamd.DBG_SPLIT, mode), ppamd.debug(ppamd.DBG_PREP_GROUP, group), \
            ppamd.debug(ppamd.DBG_SHAPE, shape):
        ppamd.evaluate(env["m"], d, prm, r, device=0)
    t.cuda.synchronize()
    return ppamd.result_to_numpy(r)


# (S, mode, parts): the automatic split (131,072 to 1,572,864 scenes) and the forced one below its
# range (more than 65,536 scenes: one K1 lane per scene); 70,013 = 17 * 4,118 + 7 leaves a partial
# last group; 1,572,865 scenes, forced: two chunks of 3 parts (split_chunks); 3,001 scenes with K1 forced to
# one lane per scene: the forced split's smallest batches (>= 2,048 scenes)
@pytest.mark.parametrize("S,mode,parts,group", [(140000, ppamd.SPLIT_AUTO, 2, 0), (420000, ppamd.SPLIT_AUTO, 3, 0),
                                                (1048583, ppamd.SPLIT_AUTO, 3, 0), (70001, ppamd.SPLIT_ON, 2, 0),
                                                (70013, ppamd.SPLIT_ON, 2, 0), (1572865, ppamd.SPLIT_ON, 6, 0),
                                                (3001, ppamd.SPLIT_ON, 2, 1)])
def test_split_bit_identical(env, S, mode, parts, group):
    sc = ppamd.synth_host(env["m"], S, seed=S, first=S)
    idx = np.arange(7, S, 211)                    # speed-edge scenes: k_cand<true> groups in both halves
    sc["ego_speed_mph"][idx] = np.array([-0.0, 5e-324, 3e6, -3.0])[np.arange(len(idx)) % 4]
    prm = ppamd.default_params()
    a = run(env, sc, prm, mode, group)
    assert ppamd.debug_get(ppamd.DBG_LAST_PARTS) == parts      # the split really ran
    b = run(env, sc, prm, ppamd.SPLIT_OFF, group)
    assert ppamd.debug_get(ppamd.DBG_LAST_PARTS) == 1
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert (x.view(np.uint8) == y.view(np.uint8)).all(), k
    edges = [S * k // d for d in (2, 3, 6) for k in range(1, d)]     # part and chunk boundaries
    sub = np.unique(np.concatenate([np.arange(0, min(300, S)), np.arange(max(S - 300, 0), S)] +
                                   [np.arange(max(e - 150, 0), min(e + 150, S)) for e in edges]))
    part = {k: np.ascontiguousarray(v[..., sub]) for k, v in sc.items()}
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], part, prm, info=False)
    got = {k: (v[:, sub] if k in ("next_x", "next_y") else v[sub]) for k, v in a.items()}
    oracle_lib.compare(got, ref)


def test_forced_split_small_batch_runs_one_stream(env):
    """Below 2,048 scenes the forced split does not run (its parts could come out empty)."""
    sc = ppamd.synth_host(env["m"], 1500, seed=9, first=9)
    prm = ppamd.default_params()
    a = run(env, sc, prm, ppamd.SPLIT_ON, 1)
    assert ppamd.debug_get(ppamd.DBG_LAST_PARTS) == 1
    b = run(env, sc, prm, ppamd.SPLIT_OFF, 1)
    for k in a:
        assert (np.asarray(a[k]).view(np.uint8) == np.asarray(b[k]).view(np.uint8)).all(), k


@pytest.mark.parametrize("S,draws,mode", [(70013, 0, ppamd.SPLIT_OFF), (140000, 0, ppamd.SPLIT_AUTO),
                                          (20011, 4, ppamd.SPLIT_OFF)])
def test_sort_cars_prepass_bit_identical(env, S, draws, mode):
    """PP_DBG_SORT_CARS 1 (round 6): k_sort_cars orders each scene's cars ahead of the one-lane K1,
    which then reads them visit-major. The values are copies in k_prep's own visiting order, so
    every output — the Frenet info, the planner's decision, paths and costs — is the gathering K1's
    bit for bit: one stream, the two-part split, and Monte-Carlo draws (per-scene order, per-draw
    noise on the original row). Round 6 measured it: K1's fetch 8.8 -> 3.0 GB per
    config-5 step, but K0 + K1 0.33 ms slower, so it is off by default."""
    t = env["torch"]
    sc = ppamd.synth_host(env["m"], S, seed=S + 7, first=S)
    idx = np.arange(5, S, 307)
    sc["ego_speed_mph"][idx] = np.array([-0.0, 5e-324, 3e6, -3.0])[np.arange(len(idx)) % 4]
    sc["car_id"][3, idx[::3]] = -1                 # the 'no car' sentinel: identity order
    sc["n_cars"][idx[1::5]] = 1                   # one row: no sort
    prm = ppamd.default_params(n_draws=draws, cost_mode=ppamd.COST_COMFORT if draws else ppamd.COST_REFERENCE)
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    out = {}
    for k0 in (1, 2):
        r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"], info=True)
        with ppamd.debug(ppamd.DBG_SPLIT, mode), ppamd.debug(ppamd.DBG_SORT_CARS, k0):
            ppamd.evaluate(env["m"], d, prm, r, device=0)
        t.cuda.synchronize()
        out[k0] = ppamd.result_to_numpy(r)
    for k in out[1]:
        a, b = np.asarray(out[1][k]), np.asarray(out[2][k])
        assert (a.view(np.uint8) == b.view(np.uint8)).all(), k

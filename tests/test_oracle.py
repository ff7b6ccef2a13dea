"""Oracle pinning (CPU): the C restatement (oracle/pp_oracle.c) against the golden vectors produced
by the reference's own code (oracle/_ref, src/main.cpp + spline.h + helpers.h) and against the
reference's DrawLines.ipynb Map::Init known-answer arrays."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

G = np.load(oracle_lib.GOLDEN + "/golden_scenes.npz")


def golden_scenes():
    return {k[len("scene_"):]: np.ascontiguousarray(G[k]) for k in G.files if k.startswith("scene_")}


def golden_params(**kw):
    return ppamd.default_params(n_speeds=int(G["n_speeds"]), speed_offsets=list(G["speed_offsets"]), **kw)


@pytest.fixture(scope="module")
def olib():
    return oracle_lib.load_oracle()


def test_map_init_matches_drawlines_kat(olib):
    """Map::Init lane centerlines vs the reference notebook's lane0..2 (4 dp => <= 5e-5)."""
    wx, wy = oracle_lib.highway_map()
    dl = np.load(oracle_lib.GOLDEN + "/drawlines_lanes.npz")
    g = np.zeros((len(wx), 10))
    assert olib.ppo_map_geometry(wx.ctypes.data_as(oracle_lib._dp), wy.ctypes.data_as(oracle_lib._dp),
                                 len(wx), g.ctypes.data_as(oracle_lib._dp)) == 0
    assert np.array_equal(np.stack([wx, wy], 1), dl["wpmap"])
    for r in range(3):
        assert np.abs(g[:, 4 + 2 * r:6 + 2 * r] - dl["lane%d" % r]).max() <= 5.0e-5 + 1e-12
    # the product's host Map::Init (pp_map_create) is bit-identical to the oracle's
    m = ppamd.Map(wx, wy)
    assert np.array_equal(m.geometry(), g)


def test_oracle_paths_bitexact_vs_reference(olib):
    wx, wy = oracle_lib.highway_map()
    sc = golden_scenes()
    r = oracle_lib.oracle_eval(olib, wx, wy, sc, golden_params(emit_paths=True))
    op = np.transpose(r["paths"], (0, 2, 1, 3))
    ref = G["ref_paths"]
    same = (op == ref) | (np.isnan(op) & np.isnan(ref))
    assert same.all()
    assert (r["path_len"] == G["ref_path_len"]).all()


def test_oracle_frame_trajectory_is_reference_choice(olib):
    """Candidate (planner lane, max_speed) reproduces the reference frame's next_x/next_y."""
    wx, wy = oracle_lib.highway_map()
    sc = golden_scenes()
    r = oracle_lib.oracle_eval(olib, wx, wy, sc, golden_params())
    ns = int(G["n_speeds"])
    assert (r["info"]["target_lane"] == G["ref_T"]).all()
    assert (r["winner"] == G["ref_T"] * ns).all()
    assert (r["n_out"] == G["ref_n"]).all()
    assert np.array_equal(np.stack([r["next_x"].T, r["next_y"].T], -1), G["ref_next"])
    info = G["ref_info"]
    assert np.array_equal(r["info"]["ego_s"], info[:, 0])
    assert np.array_equal(r["info"]["ego_d"], info[:, 1])
    assert np.array_equal(r["info"]["ego_vd"], info[:, 3])
    assert (r["info"]["ego_lane"] == info[:, 6]).all()
    assert (r["info"]["ref_wp"] == info[:, 7]).all()
    assert np.array_equal(r["cost"], G["oracle_cost"])
    assert (r["status"].view(np.uint32) == G["oracle_status"]).all()


def test_golden_covers_reference_branches():
    st = G["oracle_status"]
    for name, bit in ppamd.STATUS_BITS.items():
        if name == "NAN":
            continue
        assert np.count_nonzero(st & bit) >= 3, name


@pytest.mark.skipif(oracle_lib.load_ref() is None, reason="oracle/_ref needs /root/reference")
def test_oracle_vs_reference_large_pool(olib):
    """Fresh random + stress scenes (not stored): restatement == reference bit for bit."""
    import importlib
    import sys
    sys.path.insert(0, oracle_lib.GOLDEN)
    mg = importlib.import_module("make_golden")
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    rlib = oracle_lib.load_ref()
    offs = [-6, -4, -3, -2, -1, 0, 2]
    prm = ppamd.default_params(n_speeds=8, speed_offsets=offs, emit_paths=True)
    for sc in (ppamd.synth_host(m, 1500, seed=4242), mg.stress_pool(m, wx, wy, 1500, seed=77)[0]):
        ref = oracle_lib.ref_eval(rlib, wx, wy, sc, 8, offs)
        o = oracle_lib.oracle_eval(olib, wx, wy, sc, prm)
        op = np.transpose(o["paths"], (0, 2, 1, 3))
        assert ((op == ref["paths"]) | (np.isnan(op) & np.isnan(ref["paths"]))).all()
        assert np.array_equal(np.stack([o["next_x"].T, o["next_y"].T], -1), ref["ref_next"])

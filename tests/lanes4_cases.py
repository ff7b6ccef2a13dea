"""Four-lane parity cases (arbitrary NUM_LANES). Run by tests/test_lanes.py
in a child process whose environment selects the PP_NUM_LANES=4 builds:
  PPAMD_LIB    = carnd-path-planning-project_amd/ppamd/libppamd_l4.so  (the product, 4 lanes)
  PP_ORACLE_SO = oracle/liboracle_l4.so                                 (the restatement, 4 lanes)
  PP_REF_SO    = oracle/_ref/libppref_l4.so                             (the reference's own code
                 compiled with NUM_LANES 4: src/main.cpp:23-1154 after -DNUM_LANES=4)
The reference makes NUM_LANES a compile-time constant (src/main.cpp:22); every array, loop and
candidate count follows it, and so do ours. Same bars as the 3-lane suites: the restatement equals
the reference bit for bit; the HIP path is within 1e-6 m (oracle_lib.compare)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

OFFS = [-6, -3, -1, 0]


@pytest.fixture(scope="module")
def cpu():
    wx, wy = oracle_lib.highway_map()
    return {"m": ppamd.Map(wx, wy), "wx": wx, "wy": wy, "olib": oracle_lib.load_oracle(),
            "rlib": oracle_lib.load_ref()}


def test_builds_are_four_lane(cpu):
    assert ppamd.NUM_LANES == 4
    assert cpu["olib"].ppo_num_lanes() == 4
    prm = ppamd.default_params(n_speeds=5)
    assert ppamd.lib.pp_num_candidates(ppamd.C.byref(prm)) == 20


def test_map_init_four_lanes(cpu):
    """Host Map::Init (pp_map_create) == the restatement's, bit for bit; lane r's centre sits at
    4 (r + 0.5) m along the averaged normal (src/main.cpp:84-87, 110-129)."""
    wx, wy = cpu["wx"], cpu["wy"]
    g = np.zeros((len(wx), 12))
    assert cpu["olib"].ppo_map_geometry(wx.ctypes.data_as(oracle_lib._dp), wy.ctypes.data_as(oracle_lib._dp),
                                        len(wx), g.ctypes.data_as(oracle_lib._dp)) == 0
    got = cpu["m"].geometry()
    assert got.shape == (len(wx), 12)
    assert np.array_equal(got, g)
    c0, c3 = g[:, 4:6], g[:, 10:12]
    assert np.allclose(np.hypot(*(c3 - c0).T), 12.0, atol=0.2)


@pytest.mark.skipif(oracle_lib.load_ref() is None, reason="oracle/_ref needs /root/reference")
def test_restatement_vs_reference_four_lanes(cpu):
    """Every (lane, speed) candidate path and the frame's trajectory of the restatement equal the
    reference's own classes built with NUM_LANES 4."""
    prm = ppamd.default_params(n_speeds=len(OFFS) + 1, speed_offsets=OFFS, emit_paths=True)
    sc = ppamd.synth_host(cpu["m"], 1200, seed=4404)
    ref = oracle_lib.ref_eval(cpu["rlib"], cpu["wx"], cpu["wy"], sc, prm.n_speeds, OFFS)
    o = oracle_lib.oracle_eval(cpu["olib"], cpu["wx"], cpu["wy"], sc, prm)
    op = np.transpose(o["paths"], (0, 2, 1, 3))
    assert ((op == ref["paths"]) | (np.isnan(op) & np.isnan(ref["paths"]))).all()
    assert (o["path_len"] == ref["path_len"]).all()
    assert np.array_equal(np.stack([o["next_x"].T, o["next_y"].T], -1), ref["ref_next"])
    assert (o["info"]["target_lane"] == ref["ref_T"]).all()
    assert (o["info"]["ego_lane"] == ref["info"][:, 6]).all()
    # the fourth lane is exercised: egos in it and frames that plan into it
    assert (o["info"]["ego_lane"] == 3).sum() > 50 and (ref["ref_T"] == 3).sum() > 50


@pytest.mark.skipif(oracle_lib.load_ref() is None, reason="oracle/_ref needs /root/reference")
def test_rollout_restatement_vs_reference_four_lanes(cpu):
    sc, tr = ppamd.synth_traffic_host(cpu["m"], 6, seed=44)
    a, b = oracle_lib.copy_state(sc, tr), oracle_lib.copy_state(sc, tr)
    lo = oracle_lib.oracle_rollout(cpu["olib"], cpu["wx"], cpu["wy"], *a, ppamd.default_params(n_speeds=1),
                                   250, 3, 120.0)
    lr = oracle_lib.ref_rollout(cpu["rlib"], cpu["wx"], cpu["wy"], *b, 250, 3, 120.0)
    for k in ["ego_x", "ego_y", "ego_speed_mph", "target_lane", "n_out", "n_cars", "plan_x", "plan_y"]:
        np.testing.assert_array_equal(lo[k], lr[k], err_msg=k)
    assert (lo["target_lane"] == 3).any()


@pytest.mark.gpu
class TestFourLanesGPU:
    @pytest.fixture(scope="class")
    def env(self):
        import torch
        wx, wy = oracle_lib.highway_map()
        return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
                "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}

    @pytest.mark.parametrize("mode", [ppamd.COST_REFERENCE, ppamd.COST_COMFORT])
    def test_gpu_vs_restatement(self, env, mode):
        import test_gpu_parity as gp
        S = 3000
        prm = ppamd.default_params(n_speeds=len(OFFS) + 1, speed_offsets=OFFS, emit_paths=True, cost_mode=mode)
        d = ppamd.synth_device(env["m"], S, seed=4405 + mode, device=0)
        got = gp.run_gpu(env, d, prm, info=True)
        sc = ppamd.scenes_to_numpy(d)
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm)
        e = gp.compare(got, ref)
        assert (got["info"]["target_lane"] == ref["info"]["target_lane"]).all()
        assert (got["winner"] // prm.n_speeds == 3).sum() > 50
        print(f"4 lanes, mode {mode}: {S} scenes x {got['cost'].shape[1]} candidates, max |dxy| {e:.2e} m")

    def test_device_map_init(self, env):
        t = env["torch"]
        wx = t.from_numpy(env["wx"]).to(env["dev"])
        wy = t.from_numpy(env["wy"]).to(env["dev"])
        md = ppamd.Map.from_device(wx, wy, device=0)
        a, b = md.geometry(), env["m"].geometry()
        assert a.shape == b.shape == (len(env["wx"]), 12)
        assert np.array_equal(a, b)          # pp_glibcm.h on the device: bit for bit

    def test_gpu_rollout_vs_restatement(self, env):
        t = env["torch"]
        S, F = 256, 30
        sc, tr = ppamd.synth_traffic_host(env["m"], S, seed=46)
        a = oracle_lib.copy_state(sc, tr)
        d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
        g = {k: (t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) if isinstance(v, np.ndarray) else v)
             for k, v in tr.items()}
        prm = ppamd.default_params(n_speeds=1)
        res = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
        lg = ppamd.alloc_log(F, S, 50, xp="torch", device=env["dev"])
        ppamd.rollout(env["m"], d, g, prm, res, F, 3, 150.0, lg)
        t.cuda.synchronize()
        got = {k: x.cpu().numpy() for k, x in lg.items()}
        lo = oracle_lib.oracle_rollout(env["olib"], env["wx"], env["wy"], *a, prm, F, 3, 150.0)
        for k in ["target_lane", "n_out", "n_cars"]:
            np.testing.assert_array_equal(got[k], lo[k], err_msg=k)
        for k in ["ego_x", "ego_y", "plan_x", "plan_y"]:
            fin = np.isfinite(lo[k])
            assert (np.isfinite(got[k]) == fin).all(), k
            assert np.abs(got[k][fin] - lo[k][fin]).max() <= 1e-6, k

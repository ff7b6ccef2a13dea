"""Maps beyond highway_map.csv: any number of waypoints (above 600 the
planner reads the map from global memory instead of LDS) and Map::Init on the device."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd


def loop_map(n, a=3200.0, b=2100.0, seed=0):
    """A closed loop of n waypoints (an ellipse with a gentle wobble), counter-clockwise."""
    t = np.linspace(0, 2 * np.pi, n, endpoint=False)
    r = 1.0 + 0.02 * np.sin(5 * t + seed)
    return a * r * np.cos(t) + 1000.0, b * r * np.sin(t) - 500.0


def test_large_map_geometry_matches_oracle():
    wx, wy = loop_map(2000)
    m = ppamd.Map(wx, wy)
    g = m.geometry()
    ref = np.zeros((2000, 10))
    lib = oracle_lib.load_oracle()
    assert lib.ppo_map_geometry(np.ascontiguousarray(wx).ctypes.data_as(oracle_lib._dp),
                                np.ascontiguousarray(wy).ctypes.data_as(oracle_lib._dp), 2000,
                                ref.ctypes.data_as(oracle_lib._dp)) == 0
    assert (g.view(np.uint64) == ref.view(np.uint64)).all()


def test_degenerate_map_rejected():
    with pytest.raises(ppamd.PPError):
        ppamd.Map(np.array([0.0, 0.0, 1.0]), np.array([0.0, 0.0, 1.0]))   # zero-length segment


@pytest.mark.gpu
class TestMapsGPU:
    def test_device_map_init_matches_host(self):
        import torch
        for wx, wy in [oracle_lib.highway_map(), loop_map(5000, seed=1)]:
            host = ppamd.Map(wx, wy)
            dev = ppamd.Map.from_device(torch.from_numpy(np.ascontiguousarray(wx)).cuda(),
                                        torch.from_numpy(np.ascontiguousarray(wy)).cuda())
            # Map::Init's atan2/cos on the device are glibc's restated (pp_glibcm.h): bit for bit
            assert np.array_equal(dev.geometry(), host.geometry())

    @pytest.mark.parametrize("n", [2000, 40000])
    def test_large_map_planning_matches_oracle(self, n):
        """Scenes on a large map (global-memory map path in k_prep) against the restatement."""
        import torch
        wx, wy = loop_map(n, seed=n)
        m = ppamd.Map(wx, wy)
        from oracle_lib import compare          # the strict parity contract
        S = 3000
        sc_dev = ppamd.synth_device(m, S, seed=n, device=0)
        prm = ppamd.default_params(n_speeds=5, emit_paths=True)
        r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
        ppamd.evaluate(m, sc_dev, prm, r, device=0)
        torch.cuda.synchronize()
        got = ppamd.result_to_numpy(r)
        ref = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, ppamd.scenes_to_numpy(sc_dev), prm, info=False)
        e = compare(got, ref)
        assert e <= 1e-6, e

    @pytest.mark.parametrize("n,waves", [(300, 3), (300, 4), (2000, 3), (2000, 4)])
    def test_one_lane_k1_maps_vs_oracle(self, n, waves):
        """The one-lane K1 (PP_DBG_PREP_GROUP 1) at both builds on maps where lane matching's
        approach table (round 5, pp_device.h approach_cert) does not sit in LDS: 300 waypoints
        (the map in LDS, map and table over a block's 64 KB: k_prep<true, false> walks every
        segment exactly, the 4-wave build reads the table from global memory) and 2,000 (map and
        table in global memory)."""
        import torch
        wx, wy = loop_map(n, seed=n + waves)
        m = ppamd.Map(wx, wy)
        from oracle_lib import compare
        S = 2000
        sc_dev = ppamd.synth_device(m, S, seed=n + 17 * waves, device=0)
        prm = ppamd.default_params(n_speeds=5, emit_paths=True)
        r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
        with ppamd.debug(ppamd.DBG_PREP_GROUP, 1):
            with ppamd.debug(ppamd.DBG_PREP_WAVES, waves):
                ppamd.evaluate(m, sc_dev, prm, r, device=0)
        torch.cuda.synchronize()
        got = ppamd.result_to_numpy(r)
        ref = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, ppamd.scenes_to_numpy(sc_dev), prm, info=False)
        e = compare(got, ref)
        assert e <= 1e-6, e

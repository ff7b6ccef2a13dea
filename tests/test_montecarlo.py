"""Monte-Carlo sensor-noise mode (BASELINE config 4).

The chain that pins it:
  1. the noise generator is one definition: the library's host copy (pp_mc_gauss) and the
     oracle's C restatement agree bit for bit;
  2. a Monte-Carlo evaluation equals D independent evaluations of the materialised noisy scenes
     (per-draw costs and flags exact), and the decision is the first minimum of the
     draw-averaged cost, with the nominal (draw 0) trajectory of that candidate as output;
  3. on those noisy scenes the oracle's every candidate path equals the reference's own code
     (oracle/_ref, where it was built) bit for bit, as for the golden set;
  4. (GPU) the HIP path equals the oracle's Monte-Carlo evaluation.
"""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd


@pytest.fixture(scope="module")
def cpu():
    wx, wy = oracle_lib.highway_map()
    return {"m": ppamd.Map(wx, wy), "wx": wx, "wy": wy, "olib": oracle_lib.load_oracle(),
            "rlib": oracle_lib.load_ref()}


def test_noise_generator_host_copy_matches_oracle(cpu):
    olib = cpu["olib"]
    rng = np.random.default_rng(7)
    for _ in range(20000):
        seed = int(rng.integers(0, 2**63))
        scene = int(rng.integers(0, 2**40))
        d, j, q = int(rng.integers(1, 1024)), int(rng.integers(0, 16)), int(rng.integers(0, 4))
        a = ppamd.lib.pp_mc_gauss(seed, scene, d, j, q)
        b = olib.ppo_mc_gauss(seed, scene, d, j, q)
        assert a == b or (np.isnan(a) and np.isnan(b)), (seed, scene, d, j, q)
    g = np.array([olib.ppo_mc_gauss(0x5EED0002, s, d, j, q)
                  for s in range(40) for d in range(1, 26) for j in range(12) for q in range(4)])
    assert abs(g.mean()) < 0.02 and abs(g.std() - 1.0) < 0.02
    assert np.abs(g).max() <= 2 * np.sqrt(3) + 1e-12       # Irwin-Hall(4) support


def test_irwin_hall_integer_sum_form():
    """The library forms the noise from the integer sum of the four words (csrc/pp_synth.h
    mc_gauss: (c0 + c1 + c2 + c3 - (2^33 - 2)) (sqrt(3) 2^-32)); the oracle keeps the definition's
    form (sum of (c_i + 0.5) 2^-32, minus 2, times sqrt(3)). Every step of the definition's sum is
    exact, so both are the same product rounded once: checked on 2e6 random words and on the
    extremes."""
    rng = np.random.default_rng(11)
    c = rng.integers(0, 2**32, size=(4, 2_000_000), dtype=np.uint64).astype(np.float64)
    ext = np.array([0.0, 1.0, 2.0**31 - 1, 2.0**31, 2.0**32 - 2, 2.0**32 - 1])
    grid = np.stack(np.meshgrid(ext, ext, ext, ext, indexing="ij")).reshape(4, -1)
    c = np.concatenate([c, grid], axis=1)
    k = 1.0 / 4294967296.0
    s = (c[0] + 0.5) * k
    s = s + (c[1] + 0.5) * k
    s = s + (c[2] + 0.5) * k
    s = s + (c[3] + 0.5) * k
    old = (s - 2.0) * 1.7320508075688772
    new = (((c[0] + c[1]) + (c[2] + c[3])) - 8589934590.0) * (1.7320508075688772 * 2.0**-32)
    assert np.array_equal(old.view(np.uint64), new.view(np.uint64))


@pytest.mark.parametrize("mode,n_speeds,D", [(ppamd.COST_COMFORT, 2, 6), (ppamd.COST_REFERENCE, 1, 5)])
def test_montecarlo_equals_materialised_draws(cpu, mode, n_speeds, D):
    olib, wx, wy = cpu["olib"], cpu["wx"], cpu["wy"]
    S = 24
    sc = ppamd.synth_host(cpu["m"], S, seed=0xC0FFEE)
    prm = ppamd.default_params(n_speeds=n_speeds, cost_mode=mode, n_draws=D, noise_first_scene=1000)
    mc = oracle_lib.oracle_eval(olib, wx, wy, sc, prm)
    Cv = ppamd.NUM_LANES * n_speeds
    assert mc["cost"].shape == (S, D * Cv)
    status = np.zeros(S, np.uint32)
    nominal = None
    for d in range(D):
        nd = oracle_lib.noisy_scenes(olib, sc, prm, d)
        p1 = ppamd.default_params(n_speeds=n_speeds, cost_mode=mode, emit_paths=True)
        one = oracle_lib.oracle_eval(olib, wx, wy, nd, p1)
        np.testing.assert_array_equal(mc["cost"][:, d * Cv:(d + 1) * Cv], one["cost"])
        status |= one["status"].view(np.uint32)
        if d == 0:
            nominal = one
        if cpu["rlib"] is not None:
            ref = oracle_lib.ref_eval(cpu["rlib"], wx, wy, nd, n_speeds, [-4.0, -2.0, 0.0, 2.0][: n_speeds - 1],
                                      with_frame=False)
            op = np.transpose(one["paths"], (0, 2, 1, 3))
            assert ((op == ref["paths"]) | (np.isnan(op) & np.isnan(ref["paths"]))).all(), d
    np.testing.assert_array_equal(mc["status"].view(np.uint32), status)
    mean, win = oracle_lib.draw_decision(mc["cost"], D, Cv)
    np.testing.assert_array_equal(mc["draw_mean_cost"], mean)
    np.testing.assert_array_equal(mc["winner"], win)
    for s in range(S):
        c = win[s]
        n = nominal["path_len"][s, c]
        assert mc["n_out"][s] == n
        path = nominal["paths"][s, :n, c]
        np.testing.assert_array_equal(mc["next_x"][:n, s], path[:, 0])
        np.testing.assert_array_equal(mc["next_y"][:n, s], path[:, 1])
    if mode == ppamd.COST_REFERENCE:
        # the vote: the lane the planner picks most often across the draws wins
        Ts = np.stack([oracle_lib.oracle_eval(olib, wx, wy, oracle_lib.noisy_scenes(olib, sc, prm, d),
                                              ppamd.default_params(n_speeds=1), info=True)["info"]["target_lane"]
                       for d in range(D)], 1)
        counts = np.stack([(Ts == L).sum(1) for L in range(ppamd.NUM_LANES)], 1)
        assert (counts[np.arange(S), win // n_speeds] == counts.max(1)).all()


@pytest.mark.gpu
class TestMonteCarloGPU:
    @pytest.fixture(scope="class")
    def env(self):
        import torch
        wx, wy = oracle_lib.highway_map()
        return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
                "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}

    def run(self, env, scenes_dev, prm):
        S = int(scenes_dev["ego_x"].shape[0])
        r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
        ppamd.evaluate(env["m"], scenes_dev, prm, r, device=0)
        env["torch"].cuda.synchronize()
        return ppamd.result_to_numpy(r)

    def check(self, got, ref, D, Cv):
        """Costs within 1e-9, decisions and output counts exact, nominal trajectory within 1e-6 m,
        flags exact: every scene, no allowance."""
        np.testing.assert_allclose(got["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
        assert (got["winner"] == ref["winner"]).all()
        np.testing.assert_allclose(got["draw_mean_cost"], ref["draw_mean_cost"], rtol=1e-9, atol=1e-9)
        assert (got["n_out"] == ref["n_out"]).all()
        S = got["cost"].shape[0]
        for s in range(S):
            n = ref["n_out"][s]
            e = max(np.abs(got["next_x"][:n, s] - ref["next_x"][:n, s]).max(initial=0),
                    np.abs(got["next_y"][:n, s] - ref["next_y"][:n, s]).max(initial=0))
            assert e <= 1e-6, (s, e)
        assert (got["status"] == ref["status"].view(np.uint32)).all()

    @pytest.mark.parametrize("mode,n_speeds,D,S", [
        (ppamd.COST_REFERENCE, 1, 64, 384),     # BASELINE config 4 shape: 64 draws x 3 lanes
        (ppamd.COST_COMFORT, 1, 64, 384),
        (ppamd.COST_COMFORT, 5, 16, 160),       # C = 240: one block per scene
        (ppamd.COST_COMFORT, 5, 24, 96),        # C = 360: two blocks share a scene
        (ppamd.COST_REFERENCE, 2, 3, 700),      # several scenes per block
    ])
    def test_montecarlo_vs_oracle(self, env, mode, n_speeds, D, S):
        sc_dev = ppamd.synth_device(env["m"], S, seed=0xABCD + D, device=0)
        sc = {k: v.cpu().numpy() for k, v in sc_dev.items()}
        prm = ppamd.default_params(n_speeds=n_speeds, cost_mode=mode, n_draws=D)
        got = self.run(env, sc_dev, prm)
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
        self.check(got, ref, D, ppamd.NUM_LANES * n_speeds)

    def test_shard_offset(self, env):
        """noise_first_scene makes a shard's draws those of the same scenes in the full batch."""
        S, D = 512, 8
        sc_dev = ppamd.synth_device(env["m"], S, seed=77, device=0)
        prm = ppamd.default_params(n_speeds=1, cost_mode=ppamd.COST_COMFORT, n_draws=D)
        full = self.run(env, sc_dev, prm)
        half = {k: v[..., S // 2:].contiguous() for k, v in sc_dev.items()}
        prm2 = ppamd.default_params(n_speeds=1, cost_mode=ppamd.COST_COMFORT, n_draws=D,
                                    noise_first_scene=S // 2)
        part = self.run(env, half, prm2)
        np.testing.assert_array_equal(part["cost"], full["cost"][S // 2:])
        np.testing.assert_array_equal(part["winner"], full["winner"][S // 2:])
        np.testing.assert_array_equal(part["next_x"], full["next_x"][:, S // 2:])

"""pp_params beyond the reference's defaults (src/main.cpp:39-49: relaxed_acc, maximum_acc,
max_speed, car_length, safety_distance, keep_distance, ... are mutable globals there; the horizon
is the literal 50 at :854/:1039). Every set below is pinned to the reference's own code by
tests/test_golden_n.py (fixtures from oracle/_ref/libppref_n.so: the globals assigned per set, the
two point-count literals replaced by the set's horizon); only the cost extension (cost_mode,
costs) has no reference counterpart. Here, on 3,000 fresh scenes per set, the HIP path must equal
the restatement under the strict contract (oracle_lib.compare). k_prep's range proofs for the
unchecked divisions depend on speeds and ramp times, so the sets move those: a lower and a higher
acceleration limit, slower and
faster speed caps, shorter and longer horizons, other grids, and both cost modes. Each set also
checks that the paths-free (bench) evaluation equals the all-paths one."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

SETS = {
    "soft_acc": dict(relaxed_acc=3.0, min_relaxed_acc_while_braking=2.5, maximum_acc=5.0),
    "hard_acc": dict(relaxed_acc=8.0, min_relaxed_acc_while_braking=6.0, maximum_acc=12.0),
    "slow_cap_short": dict(max_speed=15.0, n_points=30, n_speeds=3, speed_offsets=[-3.0, 1.0]),
    "fast_cap_long": dict(max_speed=27.0, n_points=100, n_speeds=8, speed_offsets=[-6, -4, -3, -2, -1, 0, 2]),
    "spacing": dict(car_length=6.0, safety_distance=4.0, keep_distance=25.0, keep_distance_leeway=2.0),
    "comfort_hard": dict(maximum_acc=10.0, cost_mode=ppamd.COST_COMFORT, n_speeds=4, speed_offsets=[-5, -1, 3]),
    # horizon limits: 11 points (one beyond the 10 kept), 127 (the fused small-batch kernels' last
    # size), PP_MAX_POINTS = 128 (adjusted-step masks in both 64-bit words)
    "horizon_11": dict(n_points=11),
    "horizon_127": dict(n_points=127, max_speed=27.0),
    "horizon_128": dict(n_points=128, max_speed=27.0),
}
# scenes per set: 3,000 take the fused small-batch kernels where N <= 127 (k_step_small / k_cand_small);
# 20,000 at N = 128 take k_prep + k_cand + k_emit
SIZES = {"horizon_128": 20000}


def make_params(emit_paths, kw):
    kw = dict(kw)
    p = ppamd.default_params(n_speeds=kw.pop("n_speeds", 5), n_points=kw.pop("n_points", 50),
                             cost_mode=kw.pop("cost_mode", ppamd.COST_REFERENCE), emit_paths=emit_paths,
                             speed_offsets=kw.pop("speed_offsets", None))
    for k, v in kw.items():
        setattr(p, k, float(v))
    return p


def test_param_sets_are_valid_for_the_oracle():
    """CPU: every set runs through the oracle (no parameter is rejected), and the sets do change the
    decisions against the defaults on the same scenes."""
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    olib = oracle_lib.load_oracle()
    host = ppamd.synth_host(m, 200, seed=31, first=9_000_000)
    base = oracle_lib.oracle_eval(olib, wx, wy, host, make_params(True, {}), info=False)
    changed = 0
    for name, kw in SETS.items():
        r = oracle_lib.oracle_eval(olib, wx, wy, host, make_params(True, kw), info=False)
        assert r["n_out"].shape == (200,), name
        changed += int(not np.array_equal(r["status"], base["status"]) or
                       not np.allclose(r["next_x"], base["next_x"], equal_nan=True))
    assert changed == len(SETS)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SETS))
def test_param_set_vs_oracle(name):
    import torch
    kw = SETS[name]
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    olib = oracle_lib.load_oracle()
    S = SIZES.get(name, 3000)
    host = ppamd.synth_host(m, S, seed=101, first=7_000_000 + 10_000 * list(SETS).index(name))
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0") for k, v in host.items()}
    out = {}
    for paths in (True, False):
        prm = make_params(paths, kw)
        r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
        ppamd.evaluate(m, dev, prm, r, device=0)
        torch.cuda.synchronize()
        out[paths] = ppamd.result_to_numpy(r)
    ref = oracle_lib.oracle_eval(olib, wx, wy, host, make_params(True, kw), info=False)
    e = oracle_lib.compare(out[True], ref)
    got, got_e = out[False], out[True]
    np.testing.assert_array_equal(got["cost"], got_e["cost"])
    for k in ("winner", "n_out", "status"):
        assert np.array_equal(got[k], got_e[k]), (name, k)
    for k in ("next_x", "next_y"):
        e = max(e, oracle_lib.max_err(got[k], got_e[k]))
    assert e <= oracle_lib.TOL, (name, e)
    print(f"{name}: max |dxy| {e:.3e} m")


@pytest.mark.gpu
@pytest.mark.parametrize("n_points", [10, ppamd.MAX_POINTS + 1])
def test_horizon_out_of_range_rejected(n_points):
    """N must exceed the 10 kept points and stay <= PP_MAX_POINTS: PP_ERR_ARG, nothing launched"""
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    host = ppamd.synth_host(m, 64, seed=3)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0") for k, v in host.items()}
    prm = make_params(False, dict(n_points=n_points))
    r = ppamd.alloc_result(64, make_params(False, dict(n_points=min(n_points, ppamd.MAX_POINTS))),
                           xp="torch", device=torch.device("cuda", 0))
    with pytest.raises(ppamd.PPError):
        ppamd.evaluate(m, dev, prm, r, device=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n_speeds", [1, 2, 3])
def test_small_grid_fresh_batch_vs_oracle(n_speeds):
    """Small batches with C = 3, 6, 9 candidates per scene (k_step_small, whose block must hold 16
    K1 lanes per scene beside the C lanes per scene of K2). Each batch follows a different batch of
    the same size on the same stream, so no scene can reuse a prep record the previous call left in
    the workspace."""
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    olib = oracle_lib.load_oracle()
    S = 700
    prm = make_params(False, dict(n_speeds=n_speeds, speed_offsets=[-3.0, -1.0][:n_speeds - 1]))
    for first in (11_000_000, 12_000_000):
        host = ppamd.synth_host(m, S, seed=7, first=first)
        dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0") for k, v in host.items()}
        r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
        ppamd.evaluate(m, dev, prm, r, device=0)
        torch.cuda.synchronize()
    got = ppamd.result_to_numpy(r)
    ref = oracle_lib.oracle_eval(olib, wx, wy, host, prm, info=False)
    oracle_lib.compare(got, ref)

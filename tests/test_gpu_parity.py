"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors and the
CPU oracle. Tolerance (north_star): max |dxy| <= 1e-6 m per point; NaN padding identical;
integer outputs (winner, n_out, path_len, status flags) exact; costs within 1e-9 relative
(oracle_lib.compare: no allowance of any kind)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu
TOL = oracle_lib.TOL
max_err = oracle_lib.max_err
compare = oracle_lib.compare

G = np.load(oracle_lib.GOLDEN + "/golden_scenes.npz")


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def to_dev(env, d):
    return {k: env["torch"].from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in d.items()}


def run_gpu(env, scenes_dev, prm, info=False):
    S = int(scenes_dev["ego_x"].shape[0])
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"], info=info)
    ppamd.evaluate(env["m"], scenes_dev, prm, r, device=0)
    env["torch"].cuda.synchronize()
    return ppamd.result_to_numpy(r)


def compare_paths_free(env, scenes_dev, host, prm_kw, ref=None):
    """The emit_paths=False evaluation (the bench's path) against the oracle: the all-paths
    evaluation of the same scenes is compared with the oracle (compare), then the paths-free one
    with it: costs, winners, output counts and status bit for bit (the same candidate
    arithmetic), next_x/next_y within TOL (reference mode replays the winner's transform in
    k_emit); and the paths-free result with the oracle directly."""
    got_e = run_gpu(env, scenes_dev, ppamd.default_params(emit_paths=True, **prm_kw))
    if ref is None:
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host,
                                     ppamd.default_params(emit_paths=True, **prm_kw), info=False)
    e = compare(got_e, ref)
    got = run_gpu(env, scenes_dev, ppamd.default_params(emit_paths=False, **prm_kw))
    np.testing.assert_array_equal(got["cost"], got_e["cost"])
    for k in ("winner", "n_out", "status"):
        assert np.array_equal(got[k], got_e[k]), k
    for k in ("next_x", "next_y"):
        e = max(e, max_err(got[k], got_e[k]))
    assert e <= TOL, e
    ref_nopaths = {k: v for k, v in ref.items() if k not in ("paths", "path_len")}
    return max(e, compare(got, ref_nopaths))


def golden_params(**kw):
    return ppamd.default_params(n_speeds=int(G["n_speeds"]), speed_offsets=list(G["speed_offsets"]), **kw)


def test_golden_reference_vectors(env):
    """HIP vs the reference's own outputs (every candidate path + the frame's trajectory)."""
    sc = {k[6:]: G[k] for k in G.files if k.startswith("scene_")}
    got = run_gpu(env, to_dev(env, sc), golden_params(emit_paths=True), info=True)
    gp = np.transpose(got["paths"], (0, 2, 1, 3))
    e = max_err(gp, G["ref_paths"])
    assert e <= TOL, e
    assert (got["path_len"] == G["ref_path_len"]).all()
    assert (got["winner"] == G["ref_T"] * int(G["n_speeds"])).all()
    assert (got["n_out"] == G["ref_n"]).all()
    e2 = max_err(np.stack([got["next_x"].T, got["next_y"].T], -1), G["ref_next"])
    assert e2 <= TOL, e2
    assert (got["info"]["target_lane"] == G["ref_T"]).all()
    np.testing.assert_allclose(got["cost"], G["oracle_cost"], rtol=1e-9, atol=1e-9)
    assert (got["status"] == G["oracle_status"]).all()
    print(f"golden: max |dxy| paths {e:.3e} m, next {e2:.3e} m")


@pytest.mark.parametrize("mode,emit", [(ppamd.COST_REFERENCE, True), (ppamd.COST_COMFORT, True),
                                       (ppamd.COST_REFERENCE, False), (ppamd.COST_COMFORT, False)])
def test_random_scenes_vs_oracle(env, mode, emit):
    """emit=False is the bench's path: in reference mode k_cand records the winner's local path
    and k_emit writes next_x/next_y; in comfort mode k_winner re-runs the argmin candidate."""
    S = 3000
    scenes = ppamd.synth_device(env["m"], S, seed=2024, first=10**6, device=0)
    host = ppamd.scenes_to_numpy(scenes)
    if not emit:
        e = compare_paths_free(env, scenes, host, {"cost_mode": mode})
        print(f"random mode={mode} paths-free: max |dxy| {e:.3e} m")
        return
    prm = ppamd.default_params(cost_mode=mode, emit_paths=emit)
    got = run_gpu(env, scenes, prm)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    e = compare(got, ref)
    print(f"random mode={mode}: max |dxy| {e:.3e} m")


def test_tied_cars_vs_oracle(env):
    """Cars duplicated under later ids (identical position and velocity): the running minima of
    the planner and of the follow-car choice keep the earlier id, as the reference's id-order
    pass does, although k_prep visits the cars nearest class first."""
    S = 2000
    sc = ppamd.synth_host(env["m"], S, seed=77, first=4242)
    for j in range(6, 12):
        for k in ("car_x", "car_y", "car_vx", "car_vy"):
            sc[k][j] = sc[k][j - 6]
    prm = ppamd.default_params(emit_paths=True)
    got = run_gpu(env, to_dev(env, sc), prm, info=True)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=True)
    compare(got, ref)
    for k in ("in_lane_car", "target_lane", "lane_open_mask", "n_matched_cars", "ego_lane"):
        assert np.array_equal(got["info"][k], ref["info"][k]), k
    np.testing.assert_allclose(got["info"]["lane_score"], ref["info"]["lane_score"], rtol=0, atol=1e-12)
    assert (got["info"]["in_lane_car"] >= 0).sum() > S // 4


@pytest.mark.parametrize("emit", [True, False])
def test_speed_range_edges_vs_oracle(env, emit):
    """Speeds at the edges of k_cand<false>'s unchecked reciprocal divisions: telemetry speeds
    of -0, subnormal, tiny, huge and negative magnitude (frame-0 scenes take the telemetry
    speed), and a car just ahead in the ego lane whose velocity is 0, -0, subnormal or tiny (a
    LimitSpeed target of that size). k_prep routes every scene with a speed or ramp time outside
    the proven range to the checked instantiation; results must equal the oracle either way.
    (Speeds of ~1e11 m/s and more put the path at ~1e10 m, where ulp-level differences of the
    transcendentals exceed the absolute 1e-6 m tolerance: 3e6 mph = 1.3e6 m/s > 2^20 is the
    largest finite magnitude used; 1e300 mph overflows to the same non-finite path on both sides.)"""
    S = 1200
    sc = ppamd.synth_host(env["m"], S, seed=909, first=31337)
    speeds = [-0.0, 0.0, 5e-324, 1e-310, 1e-300, 1e-40, 1e-18, 2.237e-17, 1e-12, 1e-6, 0.3,
              49.66, 3e6, 1e300, -3.0, -1e-300, 2.237 * 22.2]
    vels = [0.0, -0.0, 5e-324, 1e-300, 1e-25, 1e-9, 3.0]
    p9x, p9y = sc["prev_x"][9], sc["prev_y"][9]
    hx, hy = p9x - sc["prev_x"][8], p9y - sc["prev_y"][8]
    nrm = np.maximum(np.hypot(hx, hy), 1e-12)
    for s in range(S):
        if s % 3 != 2:
            sc["n_prev"][s] = 0
            sc["ego_speed_mph"][s] = speeds[s % len(speeds)]
        if s % 2 == 0:
            sc["car_x"][0, s] = p9x[s] + hx[s] / nrm[s] * 20.0
            sc["car_y"][0, s] = p9y[s] + hy[s] / nrm[s] * 20.0
            v = vels[(s // 2) % len(vels)]
            sc["car_vx"][0, s] = v
            sc["car_vy"][0, s] = v
    if emit:
        prm = ppamd.default_params(emit_paths=True)
        got = run_gpu(env, to_dev(env, sc), prm)
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
        e = compare(got, ref)
    else:
        e = compare_paths_free(env, to_dev(env, sc), sc, {})
    print(f"speed edges (emit={emit}): max |dxy| {e:.3e} m")


@pytest.mark.parametrize("n_speeds", [4, 6, 7, 8])
def test_flat_groups_vs_oracle(env, n_speeds):
    """All-paths mode in the flat k_cand geometry (round 5, pp_eval.hip cand_geom / cand_group:
    groups of 256 consecutive candidates, scenes straddling two groups, their spline slots built in
    both and their status flags merged with atomics): C = 18, 21, 24 straddle; C = 12 keeps whole
    scenes per group. A third of the scenes carry speed-edge telemetry, so k_prep routes them to
    k_cand<true> and marks every group they touch."""
    S = 700
    sc = ppamd.synth_host(env["m"], S, seed=4100 + n_speeds, first=999)
    speeds = [-0.0, 5e-324, 1e-300, 1e-18, 3e6, -3.0]
    for s in range(0, S, 3):
        sc["n_prev"][s] = 0
        sc["ego_speed_mph"][s] = speeds[(s // 3) % len(speeds)]
    offs = [-6, -4, -3, -2, -1, 0, 2][:n_speeds - 1]
    prm = ppamd.default_params(emit_paths=True, n_speeds=n_speeds, speed_offsets=offs)
    got = run_gpu(env, to_dev(env, sc), prm)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
    e = compare(got, ref)
    print(f"flat groups, C = {3 * n_speeds}: max |dxy| {e:.3e} m")


def test_device_synth_matches_host_synth(env):
    dev = ppamd.scenes_to_numpy(ppamd.synth_device(env["m"], 2000, seed=31, first=777, device=0))
    host = ppamd.synth_host(env["m"], 2000, seed=31, first=777)
    for k in host:                    # yaw: atan2 through pp_glibcm.h on both sides
        assert np.array_equal(dev[k], host[k]), k


def test_stress_scenes_vs_oracle(env):
    import importlib
    import sys
    sys.path.insert(0, oracle_lib.GOLDEN)
    mg = importlib.import_module("make_golden")
    sc, _ = mg.stress_pool(env["m"], env["wx"], env["wy"], 3000, seed=5150)
    prm = ppamd.default_params(emit_paths=True)
    got = run_gpu(env, to_dev(env, sc), prm)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
    e = compare(got, ref)
    print(f"stress: max |dxy| {e:.3e} m")


def test_config3_horizon100_8speeds(env):
    """Config 3 shape (3 lanes x 8 speeds, 100-point horizon) against the oracle."""
    S = 1500
    offs = [-6, -4, -3, -2, -1, 0, 2]
    prm = ppamd.default_params(n_speeds=8, n_points=100, speed_offsets=offs, emit_paths=True)
    scenes = ppamd.synth_device(env["m"], S, seed=3, device=0)
    got = run_gpu(env, scenes, prm)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], ppamd.scenes_to_numpy(scenes), prm, info=False)
    e = compare(got, ref)
    print(f"config3: max |dxy| {e:.3e} m")


def test_plan_frame_is_reference_onmessage(env):
    """pp_plan_frame (one telemetry frame, host buffers) == the reference frame's next_x/next_y."""
    sc = {k[6:]: G[k] for k in G.files if k.startswith("scene_")}
    worst = 0.0
    for s in range(0, sc["ego_x"].shape[0], 7):
        nc = int(sc["n_cars"][s])
        cars = [(int(sc["car_id"][j, s]), sc["car_x"][j, s], sc["car_y"][j, s], sc["car_vx"][j, s],
                 sc["car_vy"][j, s]) for j in range(nc)][::-1]    # any order: sorted by id inside
        npv = int(sc["n_prev"][s])
        ppamd.plan_reset(env["m"])          # unrelated scenes: no car table carried over
        nx, ny, tl = ppamd.plan_frame(env["m"], sc["ego_x"][s], sc["ego_y"][s], sc["ego_yaw_deg"][s],
                                      sc["ego_speed_mph"][s], sc["prev_x"][:npv, s], sc["prev_y"][:npv, s],
                                      cars, target_lane=int(sc["prev_target_lane"][s]))
        n = int(G["ref_n"][s])
        assert len(nx) == n and tl == int(G["ref_T"][s])
        if n:
            worst = max(worst, np.abs(np.stack([nx, ny], -1) - G["ref_next"][s, :n]).max())
    assert worst <= TOL, worst


def test_edge_sizes(env):
    prm = ppamd.default_params()
    # empty batch is a no-op
    empty = ppamd.synth_device(env["m"], 1, seed=1, device=0)
    empty = {k: v[..., :0].contiguous() for k, v in empty.items()}
    r = ppamd.alloc_result(0, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], empty, prm, r, device=0)
    # ragged: sizes that do not fill a workgroup, and n_cars < car_stride with 0 cars
    for S in (1, 16, 17, 18, 255, 257):
        sc = ppamd.synth_device(env["m"], S, seed=S, device=0)
        sc["n_cars"][::2] = 0
        sc["n_cars"][1::3] = 5
        got = run_gpu(env, sc, ppamd.default_params(emit_paths=True))
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], ppamd.scenes_to_numpy(sc),
                                     ppamd.default_params(emit_paths=True), info=False)
        compare(got, ref)


def test_full_size_properties(env):
    """BASELINE config-5 batch (2,097,152 scenes x 15): deterministic, shard invariant, the
    reference decision wins in reference mode, every cost finite and bounded."""
    torch = env["torch"]
    S = 2_097_152
    prm = ppamd.default_params()
    scenes = ppamd.synth_device(env["m"], S, seed=0x5EED0001, device=0)
    r1 = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"], info=True)
    ppamd.evaluate(env["m"], scenes, prm, r1, device=0)
    r2 = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], scenes, prm, r2, device=0)
    torch.cuda.synchronize()
    for k in ("winner", "n_out", "next_x", "next_y", "cost", "status"):
        assert torch.equal(r1[k], r2[k]), k
    # shard invariance: an interior shard evaluated alone gives the same rows
    lo, hi = 1_000_003, 1_000_003 + 70_001
    sub = ppamd.synth_device(env["m"], hi - lo, seed=0x5EED0001, first=lo, device=0)
    r3 = ppamd.alloc_result(hi - lo, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], sub, prm, r3, device=0)
    torch.cuda.synchronize()
    for k in ("winner", "n_out", "cost", "status"):
        assert torch.equal(r1[k][lo:hi], r3[k]), k
    for k in ("next_x", "next_y"):
        assert torch.equal(r1[k][:, lo:hi], r3[k]), k
    info = r1["info"].cpu().numpy().view(ppamd.INFO_DTYPE).reshape(-1)
    assert torch.equal(r1["winner"].cpu(), torch.from_numpy(info["target_lane"] * 5))
    cost = r1["cost"]
    win = cost.gather(1, r1["winner"].long()[:, None])[:, 0]
    assert bool(((win >= 0) & (win <= 999)).all())
    assert bool(torch.isfinite(cost).all())
    # oracle spot check on a strided sample of the full batch
    idx = np.arange(0, S, S // 512)
    host = {k: np.ascontiguousarray(v.cpu().numpy()[..., idx]) for k, v in scenes.items()}
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    got = {k: (v[:, idx] if k.startswith("next") else v[idx])
           for k, v in ppamd.result_to_numpy({k: r1[k] for k in ("winner", "n_out", "next_x", "next_y", "cost", "status")}).items()}
    compare(got, ref)


@pytest.mark.parametrize("case", ["random", "ties_ids", "rows24", "draws"])
def test_prep_group_invariance(env, case):
    """K1 runs one lane per evaluation on large batches (cars nearest first) and a group of G lanes
    per evaluation on small ones (rows split over the group, planner in row order): every G
    (pp_debug_set(PP_DBG_PREP_GROUP, G)) gives bit-identical outputs, and G = 1 and G = 16 equal the oracle. Cases:
    random scenes; tied duplicate cars with -1, negative and large ids; 24 rows (more than one
    round per group); Monte-Carlo draws (one group per scene x draw)."""
    import test_cartable
    S = 900
    kw = {"emit_paths": True}
    if case == "rows24":
        sc = test_cartable.many_car_scenes(env["m"], S, 4321, test_cartable.ids_wide)
    else:
        sc = ppamd.synth_host(env["m"], S, seed=31, first=777)
    if case == "ties_ids":
        for j in range(6, 12):
            for k in ("car_x", "car_y", "car_vx", "car_vy"):
                sc[k][j, ::2] = sc[k][j - 6, ::2]
        sc["car_id"][:, 1::4] = (np.arange(12) * 1000 + 1000)[:, None]
        sc["car_id"][0, 3::4] = -1
    if case == "draws":
        kw = {"n_speeds": 1, "n_draws": 8, "noise_seed": 5}
    prm = ppamd.default_params(**kw)
    d = to_dev(env, sc)
    outs = {}
    try:
        for g in (1, 2, 4, 8, 16):
            ppamd.set_prep_group(g)
            outs[g] = run_gpu(env, d, prm, info=case != "draws")
    finally:
        ppamd.set_prep_group(0)
    def same(a, b):
        if a.dtype.names:
            return all(same(a[f], b[f]) for f in a.dtype.names)
        return np.array_equal(a, b, equal_nan=a.dtype.kind == "f")
    for g in (2, 4, 8, 16):
        for k, v in outs[1].items():
            assert same(outs[g][k], v), (g, k)
    if case != "draws":
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
        compare(outs[1], ref)
        compare(outs[16], ref)


@pytest.mark.parametrize("case", ["random", "speed_edges"])
def test_fused_small_invariance(env, case):
    """Reference mode without paths has three launch shapes (include/pp.h PP_DBG_SHAPE): small
    batches run the whole step in one launch (k_step_small: K1 with 16 lanes per scene, then K2 and
    K4 in the same block), or K1 then K2 + K4 in one launch (k_cand_small: the group's fast scenes,
    its flagged scenes, then the block's team computes the recorded turns' sin/cos into the freed
    spline slots and each winner lane replays its record); large batches run k_prep, k_cand<false>,
    k_cand<true> and k_emit. All give bit-identical outputs and equal the oracle. speed_edges:
    scenes flagged for the checked instantiation in most groups."""
    S = 1200
    sc = ppamd.synth_host(env["m"], S, seed=515, first=99)
    if case == "speed_edges":
        speeds = [-0.0, 5e-324, 1e-300, 1e-18, 0.3, 3e6, 1e300, -3.0]
        for s in range(0, S, 3):
            sc["n_prev"][s] = 0
            sc["ego_speed_mph"][s] = speeds[(s // 3) % len(speeds)]
    d = to_dev(env, sc)
    prm = ppamd.default_params()
    outs = {}
    for name, shape in (("k_emit", ppamd.SHAPE_SPLIT), ("k_cand_small", ppamd.SHAPE_CAND_SMALL),
                        ("step", ppamd.SHAPE_STEP)):
        with ppamd.debug(ppamd.DBG_SHAPE, shape):
            outs[name] = run_gpu(env, d, prm, info=True)
    def same(a, b):
        if a.dtype.names:
            return all(same(a[f], b[f]) for f in a.dtype.names)
        return np.array_equal(a, b, equal_nan=a.dtype.kind == "f")
    for name in ("k_cand_small", "step"):
        for k, v in outs["k_emit"].items():
            assert same(outs[name][k], v), (name, k)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
    compare(outs["step"], ref)


@pytest.mark.parametrize("case", ["random", "ties_ids", "draws"])
def test_prep_waves_invariance(env, case):
    """K1's one-lane-per-evaluation kernel has a 3- and a 4-waves-per-SIMD build (the 4-wave one is
    picked where a batch's waves fill whole rounds of 4 better, e.g. 262,144-scene shards;
    PP_DBG_PREP_WAVES forces either). Both give bit-identical outputs (scene info included) and
    equal the oracle. Cases: random scenes; tied duplicate cars with -1, negative and large ids;
    Monte-Carlo draws."""
    S = 1500
    sc = ppamd.synth_host(env["m"], S, seed=4711, first=123)
    kw = {"emit_paths": True}
    if case == "ties_ids":
        for j in range(6, 12):
            for k in ("car_x", "car_y", "car_vx", "car_vy"):
                sc[k][j, ::2] = sc[k][j - 6, ::2]
        sc["car_id"][:, 1::4] = (np.arange(12) * 1000 + 1000)[:, None]
        sc["car_id"][0, 3::4] = -1
    if case == "draws":
        kw = {"n_speeds": 1, "n_draws": 8, "noise_seed": 5}
    prm = ppamd.default_params(**kw)
    d = to_dev(env, sc)
    outs = {}
    with ppamd.debug(ppamd.DBG_PREP_GROUP, 1):          # one lane per evaluation at this size too
        for w in (3, 4):
            with ppamd.debug(ppamd.DBG_PREP_WAVES, w):
                outs[w] = run_gpu(env, d, prm, info=case != "draws")

    def same(a, b):
        if a.dtype.names:
            return all(same(a[f], b[f]) for f in a.dtype.names)
        return np.array_equal(a, b, equal_nan=a.dtype.kind == "f")
    for k, v in outs[3].items():
        assert same(outs[4][k], v), k
    if case != "draws":
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
        compare(outs[3], ref)

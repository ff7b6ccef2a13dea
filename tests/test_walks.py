"""Lane matching's approach runs (round 3, csrc/pp_device.h approach_seg / approach_walk): after the
walk's first iteration, segments on which every lane's projection is clamped to the end the walk
moves towards are walked by their clamp tests alone, and the last one before the stop is re-run in
full. The claim is bit-identity with the full walk (Map::lane_matching, src/main.cpp:199-275), so
these tests drive the cases the shortcut touches against the oracle under the strict contract:
  - cars along the lanes up to 45 waypoints (~1.7 km) ahead of and behind the ego (long forward
    and backward runs), off-centre within and beyond the lanes;
  - walks across the map's wrap (waypoint 180 -> 0 and back);
  - cars so far from the road (1e4 ... 1e7 m) that the first iteration does not improve on the
    initial 1000^2, or the per-walk bound (5e4 m) disables the runs.
The closed-loop tests (tests/test_rollout.py, tests/test_cartable.py) walk re-reported cars from a
moving ego through the same code.
Round 5: the one-lane K1 (k_prep) certifies approach segments from a per-map table by two fmas per
lane with a 1e-3 m^2 margin (approach_cert) and leaves uncertified ones to the full walk; the
grouped K1 of small batches keeps the exact test. test_certified_runs_vs_oracle forces the
one-lane K1 at both of its builds (LDS table at 3 waves per SIMD, global-memory table at 4) and adds
cars within 1e-3 m of a lane point's perpendicular, where the margin decides.
The 40,000-waypoint loop of tests/test_maps.py has lane segments shorter than 1 m: there the map
flag (fastm bit 2) turns the runs off and the full walk alone runs."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    return {"torch": torch, "m": m, "wx": wx, "wy": wy, "geo": m.geometry(),
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def to_dev(env, d):
    return {k: env["torch"].from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in d.items()}


def run_gpu(env, d, prm):
    S = int(d["ego_x"].shape[0])
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], d, prm, r, device=0)
    env["torch"].cuda.synchronize()
    return ppamd.result_to_numpy(r)


def walk_scenes(env, S, seed, far=False, edge=False):
    """Synthetic scenes whose cars sit k waypoints from the ego's nearest waypoint (k in
    [-45, 45], any lane, jittered along and across the lane); with far=True a third of the cars
    are moved 1e4 ... 1e7 m away in a random direction."""
    geo = env["geo"]
    n = geo.shape[0]
    rng = np.random.default_rng(seed)
    sc = ppamd.synth_host(env["m"], S, seed=seed, first=seed * 7919)
    J = sc["car_x"].shape[0]
    for s in range(S):
        ex, ey = sc["ego_x"][s], sc["ego_y"][s]
        w = int(np.argmin((geo[:, 0] - ex) ** 2 + (geo[:, 1] - ey) ** 2))
        for j in range(int(sc["n_cars"][s])):
            k = int(rng.integers(-45, 46))
            i = (w + k) % n
            lane = int(rng.integers(0, ppamd.NUM_LANES))
            lx, ly = geo[i, 4 + 2 * lane], geo[i, 5 + 2 * lane]
            nx, ny = geo[i, 2], geo[i, 3]
            i2 = (i + 1) % n
            tx, ty = geo[i2, 0] - geo[i, 0], geo[i2, 1] - geo[i, 1]
            tl = np.hypot(tx, ty)
            a = rng.uniform(-0.5, 0.5) * tl
            if edge and rng.random() < 0.5:      # at the lane point's perpendicular, within 1e-3 m
                a = rng.choice([0.0, 1.0, -1.0]) * 10 ** rng.uniform(-9, -3)
            off = rng.choice([rng.uniform(-1.5, 1.5), rng.uniform(-9.0, 9.0)])
            sc["car_x"][j, s] = lx + a * tx / tl + off * nx
            sc["car_y"][j, s] = ly + a * ty / tl + off * ny
            if far and rng.random() < 1 / 3:
                r, t = 10 ** rng.uniform(4, 7), rng.uniform(0, 2 * np.pi)
                sc["car_x"][j, s] = ex + r * np.cos(t)
                sc["car_y"][j, s] = ey + r * np.sin(t)
    return sc


@pytest.mark.parametrize("far", [False, True])
def test_long_walks_vs_oracle(env, far):
    S = 1500
    sc = walk_scenes(env, S, 4242 + far, far=far)
    d = to_dev(env, sc)
    for kw in ({"emit_paths": True}, {"cost_mode": ppamd.COST_COMFORT}):
        prm = ppamd.default_params(**kw)
        got = run_gpu(env, d, prm)
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
        e = oracle_lib.compare(got, ref)
        print(f"far={far} {kw}: max |dxy| {e:.3e} m")


def test_walks_across_the_wrap_vs_oracle(env):
    """Scenes whose ego sits within 20 waypoints of waypoint 0: walks of up to 45 segments cross
    the map's wrap in either direction."""
    geo = env["geo"]
    n = geo.shape[0]
    S = 3000
    sc = walk_scenes(env, S, 777)
    w = np.array([int(np.argmin((geo[:, 0] - x) ** 2 + (geo[:, 1] - y) ** 2))
                  for x, y in zip(sc["ego_x"], sc["ego_y"])])
    near = np.where((w < 20) | (w > n - 20))[0]
    assert len(near) > 50, len(near)
    sub = {k: np.ascontiguousarray(v[..., near] if v.ndim > 1 else v[near]) for k, v in sc.items()}
    d = to_dev(env, sub)
    prm = ppamd.default_params(emit_paths=True)
    got = run_gpu(env, d, prm)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sub, prm, info=False)
    e = oracle_lib.compare(got, ref)
    print(f"{len(near)} scenes near the wrap: max |dxy| {e:.3e} m")


@pytest.mark.parametrize("waves", [3, 4])
def test_certified_runs_vs_oracle(env, waves):
    """The one-lane K1 (PP_DBG_PREP_GROUP 1) at 3 waves per SIMD (the approach table in LDS) and at
    4 (in global memory), on long walks with half the cars at a lane point's perpendicular (along-
    track offsets 0 and 1e-9 ... 1e-3 m) and on walks across the wrap: bit-identical with the oracle
    (Frenet state of the ego included) and with the grouped K1, which walks every segment exactly."""
    S = 3000
    sc = walk_scenes(env, S, 9090 + waves, edge=True)
    d = to_dev(env, sc)
    prm = ppamd.default_params(emit_paths=True)
    with ppamd.debug(ppamd.DBG_PREP_GROUP, 1):
        with ppamd.debug(ppamd.DBG_PREP_WAVES, waves):
            got = run_gpu(env, d, prm)
    with ppamd.debug(ppamd.DBG_PREP_GROUP, 4):
        grp = run_gpu(env, d, prm)
    for k, v in got.items():
        w = grp[k]
        if v.dtype == np.float64:
            v, w = v.view(np.uint64), w.view(np.uint64)
        assert np.array_equal(v, w), k
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
    e = oracle_lib.compare(got, ref)
    print(f"one-lane K1 at {waves} waves, {S} scenes (cars at perpendiculars): max |dxy| {e:.3e} m")


def test_certified_runs_far_from_origin_vs_oracle(env):
    """The certified approach test's error bound grows with the coordinates' magnitude: the highway
    map moved by (+35,000, +35,000) m (lane centres up to ~3.8e4 m from the origin, inside the
    fastm bound of 4e4 that the table needs), cars at lane-point perpendiculars, the one-lane K1
    (LDS table): bit-identical with the oracle."""
    wx = np.asarray(env["wx"]) + 35000.0
    wy = np.asarray(env["wy"]) + 35000.0
    m = ppamd.Map(wx, wy)
    shifted = dict(env)
    shifted.update({"m": m, "wx": wx, "wy": wy, "geo": m.geometry()})
    S = 3000
    sc = walk_scenes(shifted, S, 5151, edge=True)
    d = to_dev(shifted, sc)
    prm = ppamd.default_params(emit_paths=True)
    with ppamd.debug(ppamd.DBG_PREP_GROUP, 1):
        got = run_gpu(shifted, d, prm)
    ref = oracle_lib.oracle_eval(env["olib"], wx, wy, sc, prm, info=False)
    e = oracle_lib.compare(got, ref)
    print(f"map at +35 km, {S} scenes (cars at perpendiculars): max |dxy| {e:.3e} m")

"""The closest-waypoint cell table (round 5; csrc/pp_eval.hip build_wgrid, csrc/pp_device.h
init_reference_waypoint): near the road k_prep reads the (at most 4) waypoints that can be the
closest one to any point of a 16 m cell instead of scanning all of them (Map::init_reference_waypoint,
src/main.cpp:150-154). The claim is bit-identity with the full scan — the first waypoint with the
smallest squared distance — so these tests put frame-0 egos (the ego position is the telemetry's)
where the table decides, against the oracle under the strict contract:
  - all along the road, up to 45 m either side of the reference line (beyond the table's 32 m
    band the scan runs), in random directions;
  - exactly on cell boundaries and one ulp either side of them (the kernel's cell index rounds);
  - on the perpendicular bisector of two waypoints (equal distances: the first index wins);
  - on waypoints themselves, and far off the road (no table: the full scan)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu

CELL, BAND = 16.0, 32.0          # build_wgrid's kCell and kNear


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": np.asarray(wx), "wy": np.asarray(wy),
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def ego_points(wx, wy, rng):
    n = len(wx)
    pts = []
    # along the road, up to 45 m off the reference line
    i = rng.integers(0, n, 3000)
    t = rng.random(3000)
    j = (i + 1) % n
    bx, by = wx[i] + (wx[j] - wx[i]) * t, wy[i] + (wy[j] - wy[i]) * t
    ang = rng.random(3000) * 2 * np.pi
    r = rng.random(3000) * 45.0
    pts.append(np.stack([bx + r * np.cos(ang), by + r * np.sin(ang)], 1))
    # cell boundaries (the table's origin: the waypoints' minimum minus 2 BAND) and one ulp off them
    x0, y0 = wx.min() - 2 * BAND, wy.min() - 2 * BAND
    k = rng.integers(0, 3000, 1000)
    px = bx[k] + r[k] * np.cos(ang[k])
    py = by[k] + r[k] * np.sin(ang[k])
    gx = x0 + np.round((px - x0) / CELL) * CELL
    gy = y0 + np.round((py - y0) / CELL) * CELL
    for dx in (-1, 0, 1):
        qx = gx if dx == 0 else np.nextafter(gx, gx + dx * np.inf)
        pts.append(np.stack([qx, py], 1))
        qy = gy if dx == 0 else np.nextafter(gy, gy + dx * np.inf)
        pts.append(np.stack([px, qy], 1))
    # the perpendicular bisector of consecutive waypoints (equal distances), and the waypoints
    i = rng.integers(0, n, 500)
    j = (i + 1) % n
    mx, my = (wx[i] + wx[j]) / 2, (wy[i] + wy[j]) / 2
    nx, ny = -(wy[j] - wy[i]), wx[j] - wx[i]
    nn = np.hypot(nx, ny)
    s = (rng.random(500) - 0.5) * 60
    pts.append(np.stack([mx + s * nx / nn, my + s * ny / nn], 1))
    pts.append(np.stack([wx, wy], 1))
    # far off the road
    pts.append(np.stack([wx.mean() + rng.normal(0, 2000, 200), wy.mean() + rng.normal(0, 2000, 200)], 1))
    return np.concatenate(pts)


def run_gpu(env, sc, prm, group, waves=0):
    """One evaluation with K1 forced to `group` lanes per scene (1: k_prep, the only K1 that reads
    the cell table; 4: k_prep_g4, which always scans) and, for group 1, `waves` per SIMD."""
    t = env["torch"]
    S = sc["ego_x"].shape[0]
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"], info=True)
    with ppamd.debug(ppamd.DBG_PREP_GROUP, group):
        with ppamd.debug(ppamd.DBG_PREP_WAVES, waves):
            ppamd.evaluate(env["m"], d, prm, r, device=0)
    t.cuda.synchronize()
    return ppamd.result_to_numpy(r)


INFO_INT = ("ref_wp", "ego_lane")
INFO_F64 = ("ego_s", "ego_d", "ref_ratio")


@pytest.mark.parametrize("waves", [3, 4])
def test_reference_waypoint_cells_vs_oracle(env, waves):
    """The batch (~9,900 scenes) would take the grouped K1 (G = 8), which never reads the table
    (ADVICE r5): K1 is forced to one lane per scene, in its 3-wave (table in LDS beside the map)
    and 4-wave (global memory) builds, and pinned bit for bit against the grouped K1's full scan."""
    rng = np.random.default_rng(2025)
    p = ego_points(env["wx"], env["wy"], rng)
    S = p.shape[0]
    sc = ppamd.synth_host(env["m"], S, seed=515, first=9000)
    sc["ego_x"][:] = p[:, 0]
    sc["ego_y"][:] = p[:, 1]
    sc["n_prev"][:] = 0                      # frame 0: the ego position is the telemetry's
    prm = ppamd.default_params(emit_paths=True)
    got = run_gpu(env, sc, prm, 1, waves)
    scan = run_gpu(env, sc, prm, 4)
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=True)
    for k in INFO_INT:
        assert np.array_equal(got["info"][k], ref["info"][k]), k
        assert np.array_equal(got["info"][k], scan["info"][k]), k
    for k in INFO_F64:
        a, b, c = got["info"][k], ref["info"][k], scan["info"][k]
        assert (a.view(np.uint64) == b.view(np.uint64)).all(), k
        assert (a.view(np.uint64) == c.view(np.uint64)).all(), k
    for k in ("winner", "n_out", "status", "path_len"):
        assert np.array_equal(got[k], scan[k]), k
    for k in ("paths", "next_x", "next_y", "cost"):
        assert (got[k].view(np.uint64) == scan[k].view(np.uint64)).all(), k
    e = oracle_lib.compare(got, ref)
    print(f"{S} egos, K1 G=1 at {waves} waves: ref_wp / Frenet state bit-identical to the oracle and "
          f"to the grouped K1's full scan, max |dxy| {e:.3e} m")

"""Parity at the BASELINE.json configurations, at their full sizes:

- config 1: one replayed telemetry frame through pp_plan_frame == the reference's own frame
  (tests/test_gpu_parity.py::test_plan_frame_is_reference_onmessage and test_cartable.py cover it);
- config 2: 4,096 scenes x 3 lanes x 5 speeds, N = 50: every candidate path of every scene
  against the restatement (strict: oracle_lib.compare), then the paths-free bench path;
- config 3: 262,144 scenes x 3 lanes x 8 speeds, N = 100, every path emitted (10 GB of paths):
  size-independent properties over the whole batch on the device (determinism, shard
  invariance, NaN padding exactly after path_len, finite points before it, the reference
  decision wins, winner path == its emitted path) plus every candidate of a strided sample of
  2,048 scenes against the restatement;
- config 4: 16,384 scenes x 64 sensor-noise draws x 3 lanes (3.1 M candidates), per-scene argmin
  over the draw-averaged cost: properties over the batch plus a strided sample of 256 scenes
  (16,384 noisy evaluations) against the restatement;
- config 5: 2,097,152 scenes (test_gpu_parity.py::test_full_size_properties, and the bench).
The restatement (oracle/pp_oracle.c) is pinned bit for bit to the reference's own code
(tests/test_oracle.py); at N = 100 too, through oracle/_ref/libppref_n.so (the reference with its
two point-count literals, src/main.cpp:854 and :1039, made settable) and the committed fixture
tests/golden/golden_config3.npz (tests/test_golden_n.py, which also tiles it into a large GPU batch)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu
OFFS8 = [-6, -4, -3, -2, -1, 0, 2]


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def run(env, scenes, prm, info=False):
    S = int(scenes["ego_x"].shape[0])
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"], info=info)
    ppamd.evaluate(env["m"], scenes, prm, r, device=0)
    env["torch"].cuda.synchronize()
    return r


def sample(d, idx):
    """host copies of rows `idx` of a scene or result dict (scene axis last, or first for
    per-scene/per-candidate arrays; next_x/next_y are point-major)"""
    out = {}
    for k, v in d.items():
        a = v.cpu().numpy() if hasattr(v, "cpu") else v
        if k in ("next_x", "next_y", "prev_x", "prev_y", "car_id", "car_x", "car_y", "car_vx", "car_vy"):
            out[k] = np.ascontiguousarray(a[..., idx])
        else:
            out[k] = np.ascontiguousarray(a[idx])
        if k == "status":
            out[k] = out[k].view(np.uint32)
    return out


def test_config2_every_candidate(env):
    S = 4096
    scenes = ppamd.synth_device(env["m"], S, seed=0x5EED0002, device=0)
    host = ppamd.scenes_to_numpy(scenes)
    prm = ppamd.default_params(emit_paths=True)
    got = ppamd.result_to_numpy(run(env, scenes, prm))
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    e = oracle_lib.compare(got, ref)
    # the bench's path (winner-only: k_cand records, k_emit replays) on the same scenes
    got2 = ppamd.result_to_numpy(run(env, scenes, ppamd.default_params()))
    ref2 = {k: v for k, v in ref.items() if k not in ("paths", "path_len")}
    e = max(e, oracle_lib.compare(got2, ref2))
    print(f"config 2: {S} x 15 candidates, max |dxy| {e:.3e} m")


def test_config3_full_size(env):
    torch = env["torch"]
    S = 262_144
    prm = ppamd.default_params(n_speeds=8, n_points=100, speed_offsets=OFFS8, emit_paths=True)
    C_, N = 24, 100
    scenes = ppamd.synth_device(env["m"], S, seed=0x5EED0003, device=0)
    r = run(env, scenes, prm)
    paths, plen = r["paths"], r["path_len"]            # [S, N, C, 2], [S, C]
    # NaN padding exactly from path_len on; finite points before it
    pt = torch.arange(N, device=env["dev"])[None, :, None]
    live = pt < plen[:, None, :]
    fin = torch.isfinite(paths).all(-1)
    nan = torch.isnan(paths).all(-1)
    assert bool((nan | live).all()), "points after path_len must be NaN"
    # (a point inside the path may be NaN only as the reference's standstill 0/0 end point)
    nan_live = (~fin & live)
    assert bool((nan_live.sum(1) <= 1).all())
    # the reference decision (planner lane, max_speed) is the winner; its path is next_x/next_y
    K = 10
    w = r["winner"].long()
    assert bool((w % 8 == 0).all())
    wp = paths[torch.arange(S, device=env["dev"]), :, w]           # [S, N, 2]
    nx = r["next_x"].T
    ny = r["next_y"].T
    n_out = r["n_out"].long()
    lv = torch.arange(N, device=env["dev"])[None, :] < n_out[:, None]
    assert bool(torch.equal(torch.where(lv, wp[..., 0], 0.0), torch.where(lv, nx, 0.0)))
    assert bool(torch.equal(torch.where(lv, wp[..., 1], 0.0), torch.where(lv, ny, 0.0)))
    assert bool((n_out == plen[torch.arange(S, device=env["dev"]), w]).all())
    # determinism and shard invariance
    lo, hi = 100_003, 100_003 + 9_001
    sub = ppamd.synth_device(env["m"], hi - lo, seed=0x5EED0003, first=lo, device=0)
    r2 = run(env, sub, prm)
    for k in ("cost", "winner", "n_out", "status", "path_len"):
        assert torch.equal(r[k][lo:hi], r2[k]), k
    assert torch.equal(torch.nan_to_num(paths[lo:hi], nan=7e7), torch.nan_to_num(r2["paths"], nan=7e7))
    del r2
    # every candidate of a strided sample against the restatement
    idx = np.arange(0, S, S // 2048)
    host = sample(scenes, idx)
    got = {k: v for k, v in sample({k: r[k] for k in ("winner", "n_out", "next_x", "next_y", "cost", "status",
                                                        "path_len")}, idx).items()}
    got["paths"] = paths[torch.from_numpy(idx).to(env["dev"])].cpu().numpy()
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    e = oracle_lib.compare(got, ref)
    print(f"config 3: {S} x {C_} candidates x {N} points emitted; sample of {len(idx)} scenes max |dxy| {e:.3e} m")
    del r, paths


def test_config4_full_size(env):
    torch = env["torch"]
    S, D = 16_384, 64
    scenes = ppamd.synth_device(env["m"], S, seed=0x5EED0004, device=0)
    for mode in (ppamd.COST_REFERENCE, ppamd.COST_COMFORT):
        prm = ppamd.default_params(n_speeds=1, n_draws=D, cost_mode=mode)
        r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
        ppamd.evaluate(env["m"], scenes, prm, r, device=0)
        torch.cuda.synchronize()
        # properties: the decision is the first minimum of the draw-averaged cost
        cv = r["cost"].view(S, D, 3)
        acc = cv[:, 0].clone()
        for d in range(1, D):                  # summed in draw order, as include/pp.h specifies
            acc = acc + cv[:, d]
        assert torch.equal(acc / D, r["draw_mean_cost"])
        first_min = torch.argmin(r["draw_mean_cost"], 1)
        assert torch.equal(first_min.int(), r["winner"])
        assert bool(torch.isfinite(r["cost"]).all())
        # strided sample against the restatement (every draw of every sampled scene)
        idx = np.arange(0, S, S // 256)
        host = sample(scenes, idx)
        got = sample({k: r[k] for k in ("winner", "n_out", "next_x", "next_y", "cost", "status", "draw_mean_cost")}, idx)
        prm_s = ppamd.default_params(n_speeds=1, n_draws=D, cost_mode=mode)
        # noise is keyed by the global scene index: evaluate each sampled scene as its own shard
        refs = []
        for j, s in enumerate(idx):
            one = {k: np.ascontiguousarray(v[..., j:j + 1]) for k, v in host.items()}
            prm_s.noise_first_scene = int(s)
            refs.append(oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], one, prm_s, info=False))
        ref = {k: (np.concatenate([x[k] for x in refs], 1) if k in ("next_x", "next_y")
                   else np.concatenate([x[k] for x in refs], 0)) for k in refs[0]}
        np.testing.assert_allclose(got["cost"], ref["cost"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(got["draw_mean_cost"], ref["draw_mean_cost"], rtol=1e-9, atol=1e-9)
        assert np.array_equal(got["winner"], ref["winner"])
        assert np.array_equal(got["n_out"], ref["n_out"])
        assert np.array_equal(got["status"], ref["status"].view(np.uint32))
        live = np.arange(50)[:, None] < got["n_out"][None, :]
        for k in ("next_x", "next_y"):
            assert oracle_lib.max_err(np.where(live, got[k], 0), np.where(live, ref[k], 0)) <= oracle_lib.TOL
        print(f"config 4 ({'reference' if mode == 0 else 'comfort'}): {S} x {D} draws x 3 lanes; "
              f"sample of {len(idx)} scenes exact decisions")

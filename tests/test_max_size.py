"""Batches whose element offsets pass 2^31, the sizes one MI355X's 288 GB of HBM holds beyond the
BASELINE configurations (maximum sizes):

- reference mode at 18,300,000 scenes x 15 candidates: the winner record k_cand writes and k_emit
  replays is 3 x 40 x S doubles (2.2e9 elements; rec_rot's offset 2 (N - K) S + g S + s passes 2^31
  in the last scenes), next_x/next_y 50 S; the comfort mode on the same batch (stored winner slots,
  k_winner_st);
- all-paths mode at 460,000 scenes x 24 candidates x 100 points: paths [((s N + i) C + c) 2] is
  2.2e9 elements.

Each batch is compared bit for bit, at windows spread over it (the last scene included), with the
same scenes evaluated as small batches of their own (synth_device(first=...): a scene is a function
of the seed and its index alone; tests/test_baseline_configs.py uses the same shard invariance at the
BASELINE sizes), and a strided sample of scenes against the restatement (oracle/pp_oracle.c)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu
OFFS8 = [-6, -4, -3, -2, -1, 0, 2]
W = 2048                                   # window size


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def run(env, scenes, prm):
    S = int(scenes["ego_x"].shape[0])
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], scenes, prm, r, device=0)
    env["torch"].cuda.synchronize()
    return r


def windows(S):
    return [0, S // 7, S // 2 + 7, S - 3 * W - 11, S - W]


def check_windows(env, r, S, seed, prm, keys):
    torch = env["torch"]
    for lo in windows(S):
        hi = lo + W
        sub = ppamd.synth_device(env["m"], W, seed=seed, first=lo, device=0)
        r2 = run(env, sub, prm)
        for k in keys:
            if k in ("next_x", "next_y"):
                a, b = r[k][:, lo:hi], r2[k]
            else:
                a, b = r[k][lo:hi], r2[k]
            assert torch.equal(torch.nan_to_num(a, nan=7e7) if a.is_floating_point() else a,
                               torch.nan_to_num(b, nan=7e7) if b.is_floating_point() else b), (k, lo)
        del r2, sub


def sample(d, idx):
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


def test_reference_and_comfort_beyond_2g_elements(env):
    torch = env["torch"]
    S, seed = 18_300_000, 0x5EED0006
    assert 3 * 40 * S > 2**31
    scenes = ppamd.synth_device(env["m"], S, seed=seed, device=0)
    idx = np.concatenate([np.arange(0, S, S // 256), np.arange(S - 64, S)])
    host = sample(scenes, idx)
    keys = ("next_x", "next_y", "cost", "winner", "n_out", "status")
    for mode in (ppamd.COST_REFERENCE, ppamd.COST_COMFORT):
        prm = ppamd.default_params(cost_mode=mode)
        r = run(env, scenes, prm)
        n_out = r["n_out"]
        assert bool((n_out >= 1).all()) and bool((n_out <= 50).all())
        check_windows(env, r, S, seed, prm, keys)
        got = sample({k: r[k] for k in keys}, idx)
        del r
        torch.cuda.empty_cache()
        ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
        e = oracle_lib.compare(got, ref)
        print(f"{S} scenes, cost mode {mode}: {len(windows(S))} windows of {W} bit-identical to their own "
              f"batches; {len(idx)} sampled scenes max |dxy| {e:.3e} m")
    del scenes
    torch.cuda.empty_cache()


def test_all_paths_beyond_2g_elements(env):
    torch = env["torch"]
    S, seed = 460_000, 0x5EED0007
    N, C_ = 100, 24
    assert S * N * C_ * 2 > 2**31
    prm = ppamd.default_params(n_speeds=8, n_points=N, speed_offsets=OFFS8, emit_paths=True)
    scenes = ppamd.synth_device(env["m"], S, seed=seed, device=0)
    r = run(env, scenes, prm)
    check_windows(env, r, S, seed, prm, ("paths", "path_len", "cost", "winner", "n_out", "status",
                                         "next_x", "next_y"))
    idx = np.concatenate([np.arange(0, S, S // 128), np.arange(S - 32, S)])
    host = sample(scenes, idx)
    got = sample({k: r[k] for k in ("winner", "n_out", "next_x", "next_y", "cost", "status", "path_len")}, idx)
    got["paths"] = r["paths"][torch.from_numpy(idx).to(env["dev"])].cpu().numpy()
    del r, scenes
    torch.cuda.empty_cache()
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    e = oracle_lib.compare(got, ref)
    print(f"{S} scenes x {C_} x {N} points: windows bit-identical; {len(idx)} sampled scenes max |dxy| {e:.3e} m")

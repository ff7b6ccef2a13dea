"""pp_eval's two-stream pipeline (large reference-mode batches): K2 runs chunk after chunk on the
caller's stream while a second stream runs K1 of the next chunk and K4 of the previous one. The
chunks use the same kernels over group ranges, so every output must equal the one-chunk launch
bit for bit — including scenes that k_prep routes to k_cand<true> (each chunk keeps its own
flagged-group list) — and the chunked result must match the oracle on a strided sample."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint64) if a.dtype == np.float64 else a


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


def edge_scenes(env, S, seed):
    """Synthetic scenes with speed-edge scenes (k_cand<true>) spread over the whole batch."""
    sc = ppamd.synth_host(env["m"], S, seed=seed, first=5 * 10**6)
    speeds = [-0.0, 5e-324, 1e-300, 1e-40, 3e6, 1e300, -3.0]
    idx = np.arange(0, S, 997)
    sc["n_prev"][idx] = 0
    sc["ego_speed_mph"][idx] = np.array(speeds)[np.arange(len(idx)) % len(speeds)]
    return sc, idx


def run(env, scenes_dev, S, chunks, monkeypatch):
    monkeypatch.setenv("PP_CHUNKS", str(chunks))
    prm = ppamd.default_params()
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], scenes_dev, prm, r, device=0)
    env["torch"].cuda.synchronize()
    return ppamd.result_to_numpy(r)


def test_pipeline_chunks_bit_identical(env, monkeypatch):
    S = 200_003                                   # not a multiple of the group or chunk size
    sc, idx = edge_scenes(env, S, seed=4711)
    dev = {k: env["torch"].from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    base = run(env, dev, S, 1, monkeypatch)
    assert (base["status"][idx] != 0).any()
    for chunks in (2, 3, 5, 8, 16):
        got = run(env, dev, S, chunks, monkeypatch)
        for k in ("winner", "n_out", "status", "cost", "next_x", "next_y"):
            assert np.array_equal(bits(got[k]), bits(base[k])), (chunks, k)
    # the chunked result against the oracle: the flagged scenes and a strided sample
    samp = np.unique(np.concatenate([idx, np.arange(5, S, 1601)]))
    host = {k: np.ascontiguousarray(v[..., samp]) for k, v in sc.items()}
    prm = ppamd.default_params()
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], host, prm, info=False)
    sub = {k: got[k][samp] for k in ("winner", "n_out", "status", "cost")}
    sub.update({k: got[k][:, samp] for k in ("next_x", "next_y")})     # point-major [N][S]
    e = oracle_lib.compare(sub, ref)
    print(f"pipeline: {len(samp)} sampled scenes vs oracle, max |dxy| {e:.3e} m")

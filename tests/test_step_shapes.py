"""The one-launch step (k_step_small, reference mode, batches up to 16,384 scenes) in each of its
block shapes (pp_eval: step_waves_on), against the restatement, with speed-edge scenes that route
groups to the checked pass:
  - up to 2,048 scenes (8-scene blocks fit one per CU): 256 threads, K1 on waves 0-1 beside phase A
    on waves 2-3 (wave_step_body<256>, also the frame kernel's body);
  - up to 4,096 scenes (16-scene blocks fit one per CU): 512 threads (k_step_small512);
  - beyond: 16-scene blocks of 256 threads, K1 then phase A (step_small_body).
Sizes on either side of each bound; large batches are checked on the block-boundary scenes and a
strided sample (scenes are independent, so a sample is a batch of its own for the oracle)."""
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy,
            "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}


@pytest.mark.parametrize("S", [1, 7, 8, 9, 2047, 2048, 2049, 4095, 4096, 4097, 9000])
def test_step_block_shapes_vs_oracle(env, S):
    t = env["torch"]
    sc = ppamd.synth_host(env["m"], S, seed=S + 17, first=S * 3)
    idx = np.arange(2, S, 37)
    sc["ego_speed_mph"][idx] = np.array([-0.0, 5e-324, 3e6, -3.0])[np.arange(len(idx)) % 4]
    prm = ppamd.default_params()
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    with ppamd.debug(ppamd.DBG_SHAPE, ppamd.SHAPE_STEP):
        ppamd.evaluate(env["m"], d, prm, r, device=0)
    t.cuda.synchronize()
    got = ppamd.result_to_numpy(r)
    if S <= 64:
        sub = np.arange(S)
    else:
        edges = np.concatenate([np.arange(b - 2, b + 2) for b in range(8, S, 8)])
        sub = np.unique(np.concatenate([edges[(edges >= 0) & (edges < S)][::7], np.arange(0, S, 13), [S - 1]]))
    part = {k: np.ascontiguousarray(v[..., sub]) for k, v in sc.items()}
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], part, prm, info=False)
    sel = {k: (v[:, sub] if k in ("next_x", "next_y") else v[sub]) for k, v in got.items()}
    oracle_lib.compare(sel, ref)

"""The multi-stream split (pp_eval, include/pp.h PP_DBG_SPLIT): reference-mode batches of about a
2-, 4- or 8-GPU shard's size run as 2 parts (up to 393,216 scenes) or 3 parts, each K1 -> K2 -> K4 on
its own stream. The parts write disjoint ranges of every buffer and keep separate flagged-group
lists, so the results must be the one-stream launch's BIT FOR BIT, including the scenes routed to
k_cand<true> and part boundaries that split no group; a sample is checked against the oracle."""
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


def run(env, sc, prm, mode):
    t = env["torch"]
    S = sc["ego_x"].shape[0]
    d = {k: t.from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    with ppamd.debug(ppamd.DBG_SPLIT, mode):
        ppamd.evaluate(env["m"], d, prm, r, device=0)
    t.cuda.synchronize()
    return ppamd.result_to_numpy(r)


# (S, mode, parts): the automatic split (131,072 to 1,572,864 scenes) and the forced one below its
# range (more than 65,536 scenes: one K1 lane per scene); 70,013 = 17 * 4,118 + 7 leaves a partial
# last group
@pytest.mark.parametrize("S,mode,parts", [(140000, ppamd.SPLIT_AUTO, 2), (420000, ppamd.SPLIT_AUTO, 3),
                                          (1048583, ppamd.SPLIT_AUTO, 3), (70001, ppamd.SPLIT_ON, 2),
                                          (70013, ppamd.SPLIT_ON, 2)])
def test_split_bit_identical(env, S, mode, parts):
    sc = ppamd.synth_host(env["m"], S, seed=S, first=S)
    idx = np.arange(7, S, 211)                    # speed-edge scenes: k_cand<true> groups in both halves
    sc["ego_speed_mph"][idx] = np.array([-0.0, 5e-324, 3e6, -3.0])[np.arange(len(idx)) % 4]
    prm = ppamd.default_params()
    a = run(env, sc, prm, mode)
    assert ppamd.debug_get(ppamd.DBG_LAST_PARTS) == parts      # the split really ran
    b = run(env, sc, prm, ppamd.SPLIT_OFF)
    assert ppamd.debug_get(ppamd.DBG_LAST_PARTS) == 1
    for k in a:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert (x.view(np.uint8) == y.view(np.uint8)).all(), k
    sub = np.unique(np.r_[0:300, S // 3 - 200:S // 3 + 200, S // 2 - 300:S // 2 + 300, 2 * S // 3 - 200:2 * S // 3 + 200,
                          S - 300:S])
    part = {k: np.ascontiguousarray(v[..., sub]) for k, v in sc.items()}
    ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], part, prm, info=False)
    got = {k: (v[:, sub] if k in ("next_x", "next_y") else v[sub]) for k, v in a.items()}
    oracle_lib.compare(got, ref)

"""Generate the golden fixtures that pin BASELINE config 3 (N = 100, 8 speeds) and the non-default
pp_params sets to the reference's own code (run in the build container, where /root/reference
exists, after `make -C oracle`). Committed together with its outputs; the GPU box only reads the
.npz files.

The reference's tunables (src/main.cpp:39-49) are mutable globals: oracle/ref_harness.cpp
ref_set_params assigns them. Its horizon is two point-count literals (:854, :1039):
oracle/_ref/libppref_n.so is the reference with exactly those two replaced by a settable count
(oracle/Makefile), so N = 100 and the other horizons run through the reference's own classes.

Outputs
- golden_config3.npz: BASELINE config 3's parameters (N = 100, speeds = max_speed and ego speed
  + {-6, -4, -3, -2, -1, 0, +2}), about 170 scenes: random scenes of the bench distribution plus
  branch-coverage scenes picked greedily by status flag from a stress pool.
- golden_params.npz: every parameter set of tests/test_params.py (SETS), about 40 scenes each,
  chosen the same way; keys "<set>__<field>", the set's keyword arguments as JSON in "<set>__kw".
Each holds the scene inputs, the reference's outputs (every candidate path and its length, the
frame's own trajectory, its target lane and ego state) and the C restatement's costs, winners and
status words (the cost is this library's extension; it has no reference counterpart). The
script asserts restatement == reference bit for bit before writing.

Usage: python tests/golden/make_golden_n.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402
import make_golden  # noqa: E402  (stress_pool, take)
import test_params  # noqa: E402  (SETS, make_params)

CONFIG3 = dict(n_points=100, n_speeds=8, speed_offsets=[-6, -4, -3, -2, -1, 0, 2])


def pick_scenes(m, wx, wy, olib, prm, n_rand, per_flag, per_kind, seed):
    """Random scenes + a greedy branch-covering subset of a stress pool (status flags and every
    stress kind of make_golden.stress_pool)."""
    rand = ppamd.synth_host(m, n_rand, seed=seed, first=seed * 1000)
    pool, kind = make_golden.stress_pool(m, wx, wy, 3000, seed=seed + 1)
    st = oracle_lib.oracle_eval(olib, wx, wy, pool, prm, info=False)["status"].view(np.uint32)
    picked = []
    for name, bit in ppamd.STATUS_BITS.items():
        for i in np.nonzero(st & bit)[0][:per_flag]:
            if int(i) not in picked:
                picked.append(int(i))
    for kk in range(9):
        for i in np.nonzero(kind == kk)[0][:per_kind]:
            if int(i) not in picked:
                picked.append(int(i))
    cov = make_golden.take(pool, np.array(picked))
    return {k: np.ascontiguousarray(np.concatenate([rand[k], cov[k]], axis=-1)) for k in rand}


def pinned(olib, rlib, wx, wy, scenes, prm):
    """Reference and restatement on the same scenes; asserts bit-exact paths and frame trajectory."""
    ref = oracle_lib.ref_eval(rlib, wx, wy, scenes, prm=prm)
    o = oracle_lib.oracle_eval(olib, wx, wy, scenes, prm)
    op = np.transpose(o["paths"], (0, 2, 1, 3))
    same = (op == ref["paths"]) | (np.isnan(op) & np.isnan(ref["paths"]))
    assert same.all(), f"oracle != reference on {np.count_nonzero(~same)} values"
    assert (o["path_len"] == ref["path_len"]).all()
    assert (o["info"]["target_lane"] == ref["ref_T"]).all()
    if prm.cost_mode == ppamd.COST_REFERENCE:    # the winner is the reference frame's trajectory
        assert (o["n_out"] == ref["ref_n"]).all()
        wn = np.stack([o["next_x"].T, o["next_y"].T], -1)
        assert (wn == ref["ref_next"]).all()
    out = {"scene_" + k: v for k, v in scenes.items()}
    out.update(ref_next=ref["ref_next"], ref_n=ref["ref_n"], ref_T=ref["ref_T"], ref_paths=ref["paths"],
               ref_path_len=ref["path_len"], ref_info=ref["info"], oracle_cost=o["cost"],
               oracle_winner=o["winner"], oracle_status=o["status"].view(np.uint32),
               oracle_n_out=o["n_out"], oracle_next_x=o["next_x"], oracle_next_y=o["next_y"])
    return out


def main():
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    olib = oracle_lib.load_oracle()
    rlib = oracle_lib.load_ref_n()
    assert rlib is not None, "build oracle/_ref first: make -C oracle"

    prm = test_params.make_params(True, CONFIG3)
    sc = pick_scenes(m, wx, wy, olib, prm, n_rand=120, per_flag=6, per_kind=3, seed=303)
    g = pinned(olib, rlib, wx, wy, sc, prm)
    g["kw"] = np.array(json.dumps(CONFIG3))
    np.savez_compressed(os.path.join(HERE, "golden_config3.npz"), **g)
    S = sc["ego_x"].shape[0]
    print(f"config 3: oracle == reference (bit-exact) on {S} scenes x {3 * prm.n_speeds} candidates, N = 100")
    flags = g["oracle_status"]
    print("  flags covered:", [n for n, b in ppamd.STATUS_BITS.items() if np.count_nonzero(flags & b)])

    allp = {}
    for i, (name, kw) in enumerate(test_params.SETS.items()):
        prm = test_params.make_params(True, kw)
        sc = pick_scenes(m, wx, wy, olib, prm, n_rand=16, per_flag=2, per_kind=1, seed=400 + 10 * i)
        g = pinned(olib, rlib, wx, wy, sc, prm)
        kwj = {k: (int(v) if k == "cost_mode" else v) for k, v in kw.items()}
        g["kw"] = np.array(json.dumps(kwj))
        allp.update({f"{name}__{k}": v for k, v in g.items()})
        print(f"{name}: oracle == reference (bit-exact) on {sc['ego_x'].shape[0]} scenes x "
              f"{3 * prm.n_speeds} candidates, N = {prm.n_points}")
    np.savez_compressed(os.path.join(HERE, "golden_params.npz"), **allp)


if __name__ == "__main__":
    main()

"""BASELINE config 3 (N = 100, 8 speeds) and every non-default pp_params set, pinned to the
reference's own code.

The fixtures (tests/golden/golden_config3.npz, golden_params.npz; made by
tests/golden/make_golden_n.py) hold the outputs of oracle/_ref/libppref_n.so: the reference's
src/main.cpp:22-1154 with its tunable globals (:39-49) assigned per set (ref_set_params) and its
two point-count literals (:854, :1039) replaced by the set's horizon. CPU: the restatement equals
them bit for bit (and, where /root/reference exists, a fresh pool run through the reference
live). GPU: the HIP path equals them under the strict contract (every path point and next_x/next_y
within 1e-6 m with an identical NaN pattern, path lengths, winners, output counts and status
words exact, costs within 1e-9 against the restatement's: the cost is this library's extension)."""
import json

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd
import test_params

G3 = np.load(oracle_lib.GOLDEN + "/golden_config3.npz")
GP = np.load(oracle_lib.GOLDEN + "/golden_params.npz")
SETS = sorted({k.split("__")[0] for k in GP.files})


def fixture(name):
    """(scenes, fields, kw) of the config-3 fixture (name "config3") or of one parameter set."""
    if name == "config3":
        f = {k: G3[k] for k in G3.files}
    else:
        f = {k.split("__", 1)[1]: GP[k] for k in GP.files if k.startswith(name + "__")}
    sc = {k[len("scene_"):]: np.ascontiguousarray(v) for k, v in f.items() if k.startswith("scene_")}
    return sc, f, json.loads(str(f["kw"]))


CASES = ["config3"] + SETS


def test_fixture_sets_are_test_params_sets():
    """The fixture was made from exactly the parameter sets tests/test_params.py runs."""
    assert set(SETS) == set(test_params.SETS)
    for name in SETS:
        kw = fixture(name)[2]
        assert kw == json.loads(json.dumps(test_params.SETS[name])), name


def check_vs_reference(got, f, prm, tol):
    """got (numpy pp_result, emit_paths) against the reference fields of fixture f."""
    gp = np.transpose(got["paths"], (0, 2, 1, 3))          # [S][C][N][2]
    if tol == 0:
        same = (gp == f["ref_paths"]) | (np.isnan(gp) & np.isnan(f["ref_paths"]))
        assert same.all(), f"{np.count_nonzero(~same)} path values differ from the reference"
        e = 0.0
    else:
        e = oracle_lib.max_err(gp, f["ref_paths"])
        assert e <= tol, e
    assert (got["path_len"] == f["ref_path_len"]).all()
    if prm.cost_mode == ppamd.COST_REFERENCE:
        ns = prm.n_speeds
        assert (got["winner"] == f["ref_T"] * ns).all()
        assert (got["n_out"] == f["ref_n"]).all()
        wn = np.stack([got["next_x"].T, got["next_y"].T], -1)
        live = np.arange(wn.shape[1])[None, :, None] < f["ref_n"][:, None, None]
        e2 = oracle_lib.max_err(np.where(live, wn, 0.0), np.where(live, f["ref_next"], 0.0))
        assert e2 <= tol, e2
        e = max(e, e2)
    return e


@pytest.mark.parametrize("name", CASES)
def test_restatement_equals_reference_fixture(name):
    """CPU: the C restatement reproduces the reference's outputs bit for bit, and its own stored
    costs, winners and status words exactly."""
    wx, wy = oracle_lib.highway_map()
    sc, f, kw = fixture(name)
    prm = test_params.make_params(True, kw)
    o = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, sc, prm)
    check_vs_reference(o, f, prm, tol=0)
    assert (o["info"]["target_lane"] == f["ref_T"]).all()
    assert np.array_equal(o["info"]["ego_s"], f["ref_info"][:, 0])
    assert np.array_equal(o["cost"], f["oracle_cost"])
    assert (o["winner"] == f["oracle_winner"]).all()
    assert (o["status"].view(np.uint32) == f["oracle_status"]).all()


def test_config3_fixture_covers_reference_branches():
    st = G3["oracle_status"]
    for name, bit in ppamd.STATUS_BITS.items():
        if name == "NAN":
            continue
        assert np.count_nonzero(st & bit) >= 3, name
    assert int(G3["ref_path_len"].max()) == 100 and G3["ref_paths"].shape[2] == 100


@pytest.mark.skipif(oracle_lib.load_ref_n() is None, reason="oracle/_ref needs /root/reference")
@pytest.mark.parametrize("name", ["config3", "fast_cap_long", "hard_acc", "spacing", "horizon_128"])
def test_restatement_vs_reference_live(name):
    """Fresh scenes (not stored), through the reference's own code: bit for bit."""
    import sys
    if oracle_lib.GOLDEN not in sys.path:
        sys.path.insert(0, oracle_lib.GOLDEN)
    import make_golden
    import make_golden_n
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    kw = make_golden_n.CONFIG3 if name == "config3" else test_params.SETS[name]
    prm = test_params.make_params(True, kw)
    rlib = oracle_lib.load_ref_n()
    olib = oracle_lib.load_oracle()
    for sc in (ppamd.synth_host(m, 400, seed=8080), make_golden.stress_pool(m, wx, wy, 400, seed=8081)[0]):
        make_golden_n.pinned(olib, rlib, wx, wy, sc, prm)     # asserts bit-exact


@pytest.mark.skipif(oracle_lib.load_ref_n() is None, reason="oracle/_ref needs /root/reference")
def test_horizon_build_equals_pristine_reference_at_50():
    """The line-substituted reference at N = 50 is the pristine reference build, bit for bit; the
    pristine build refuses any other horizon."""
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    sc = ppamd.synth_host(m, 300, seed=99)
    offs = [-4.0, -2.0, 0.0, 2.0]
    a = oracle_lib.ref_eval(oracle_lib.load_ref_n(), wx, wy, sc, 5, offs)
    b = oracle_lib.ref_eval(oracle_lib.load_ref(), wx, wy, sc, 5, offs)
    for k in ("paths", "ref_next"):
        assert np.array_equal(a[k], b[k], equal_nan=True), k
    assert np.array_equal(a["path_len"], b["path_len"])
    import ctypes as C
    p = ppamd.default_params(n_points=100)
    assert oracle_lib.load_ref().ref_set_params(C.byref(p)) == -1


def tile(sc, f, reps):
    """The fixture repeated `reps` times along the scene axis (point-major inputs [i][s] tile on
    their last axis, per-scene outputs on their first)."""
    sc = {k: np.ascontiguousarray(np.tile(v, reps) if v.ndim == 1 else np.tile(v, (1, reps)))
          for k, v in sc.items()}
    f = dict(f)
    for k in ("ref_paths", "ref_path_len", "ref_T", "ref_n", "ref_next", "oracle_cost", "oracle_winner",
              "oracle_status", "oracle_n_out"):
        f[k] = np.tile(f[k], (reps,) + (1,) * (f[k].ndim - 1))
    for k in ("oracle_next_x", "oracle_next_y"):
        f[k] = np.tile(f[k], (1, reps))
    return sc, f


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
@pytest.mark.parametrize("name", CASES)
def test_gpu_vs_reference_fixture(name, tiled):
    """The HIP path against the reference's outputs: the all-paths evaluation (every candidate path
    vs the reference, then the whole result under oracle_lib.compare against the restatement's
    stored outputs) and the paths-free evaluation (the bench's path: the same costs, winners and
    status bit for bit, next_x/next_y within 1e-6 m of the reference frame's trajectory).
    The fixture alone is a small batch (the fused kernels k_step_small / k_cand_small where
    N <= 127); tiled to more than 16,384 scenes it runs k_prep + k_cand + k_emit, the large-batch
    kernels of BASELINE config 3 itself."""
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    sc, f, kw = fixture(name)
    if tiled:
        sc, f = tile(sc, f, -(-20000 // sc["ego_x"].shape[0]))
    S = sc["ego_x"].shape[0]
    dev = {k: torch.from_numpy(v).to("cuda:0") for k, v in sc.items()}
    out = {}
    for paths in (True, False):
        prm = test_params.make_params(paths, kw)
        r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
        ppamd.evaluate(m, dev, prm, r, device=0)
        torch.cuda.synchronize()
        out[paths] = ppamd.result_to_numpy(r)
    prm = test_params.make_params(True, kw)
    e = check_vs_reference(out[True], f, prm, tol=oracle_lib.TOL)
    ref = {"winner": f["oracle_winner"], "n_out": f["oracle_n_out"], "next_x": f["oracle_next_x"],
           "next_y": f["oracle_next_y"], "cost": f["oracle_cost"], "status": f["oracle_status"]}
    e = max(e, oracle_lib.compare(out[True], ref))
    got = out[False]
    np.testing.assert_array_equal(got["cost"], out[True]["cost"])
    for k in ("winner", "n_out", "status"):
        assert np.array_equal(got[k], out[True][k]), k
    e = max(e, oracle_lib.compare(got, ref))
    print(f"{name}: {S} scenes, max |dxy| vs reference {e:.3e} m")

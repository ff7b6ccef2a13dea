"""Whole-batch parity at every BASELINE GPU configuration, with a near-threshold census
("the parity test reports the worst scene, the
count above 1e-6, and a near-threshold flag").

For configs 5 (2,097,152 scenes x 15 candidates; in the reference decision and, as "5c", in the
comfort cost mode's per-scene argmin), 3 (262,144 x 24, 100 points, every path) and 4 (16,384 x
64 sensor-noise draws x 3 lanes) the HIP product path evaluates the whole BASELINE batch
and EVERY scene is compared with the C restatement (oracle/pp_oracle.c, run over the same host
scenes on 16 threads) under the strict contract of oracle_lib.compare: winners, output counts,
path lengths and status words exact, every path point and next_x/next_y within 1e-6 m with an
identical NaN pattern, costs within 1e-9 relative. The report per config:
  - the worst |dxy| and the scene holding it, and the count of points above 1e-6 m (must be 0);
  - the oracle's limiter decisions (src/main.cpp:941 and :972) and how many of them lie within a
    relative 1e-12 of maximum_acc (oracle/pp_oracle.c ppo_census);
  - from the -DPP_LIMCENSUS build (tools/limit_census.py, a child process on the same scenes):
    the decisions where the kernel's operation sequence (asin of the unit-step cross product,
    Markstein-corrected divisions) and the reference's (glibc atan2 differences, IEEE divisions)
    decide differently, and the near-threshold decisions seen on the GPU.
Every report line is printed and written to gpurun_out/full_batch_census.json (copied into
profiles/ per round)."""
import json
import os
import subprocess
import sys
import threading
import time

import ctypes as C
import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu

REPO = oracle_lib.REPO
CENSUS_LIB = os.path.join(oracle_lib.PKG, "ppamd", "libppamd_census.so")
OUT = os.path.join(REPO, "gpurun_out", "full_batch_census.json")
THREADS = 16                           # the GPU box's CPU share for one GPU
CONFIGS = {5: dict(S=2097152, ns=5, N=50, paths=False, draws=0),
           3: dict(S=262144, ns=8, N=100, paths=True, draws=0),
           4: dict(S=16384, ns=1, N=50, paths=False, draws=64),
           # config 5's batch in the comfort cost mode: the per-scene argmin of the candidate costs,
           # taken in k_cand's block, and the winner re-run by k_winner_st from its stored spline
           "5c": dict(S=2097152, ns=5, N=50, paths=False, draws=0, comfort=True)}


def params(cfg):
    return ppamd.default_params(n_speeds=cfg["ns"], n_points=cfg["N"], emit_paths=cfg["paths"],
                                n_draws=cfg["draws"], noise_first_scene=0,
                                cost_mode=ppamd.COST_COMFORT if cfg.get("comfort") else ppamd.COST_REFERENCE,
                                speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if cfg["ns"] == 8 else None)


def oracle_full(olib, wx, wy, host, prm, threads=THREADS, chunk=4096):
    """The restatement over every scene: worker threads take chunks of one shared result (ctypes
    releases the GIL), each summing its thread's limiter census."""
    olib.ppo_census.argtypes = [C.POINTER(C.c_longlong), C.c_int]
    S = int(host["ego_x"].shape[0])
    r = ppamd.alloc_result(S, prm, info=False)
    if prm.emit_paths:
        r["paths"][:] = np.nan
    b = ppamd.scene_struct(host)
    R = ppamd.result_struct(r)
    wxa = np.ascontiguousarray(wx, np.float64)
    wya = np.ascontiguousarray(wy, np.float64)
    dp = C.POINTER(C.c_double)
    lock = threading.Lock()
    state = {"next": 0, "census": np.zeros(4, np.int64), "rc": 0}

    def worker():
        cen = (C.c_longlong * 4)()
        olib.ppo_census(cen, 1)                   # this thread's counters from zero
        while True:
            with lock:
                lo = state["next"]
                state["next"] += chunk
            if lo >= S:
                break
            rc = olib.ppo_eval_range(wxa.ctypes.data_as(dp), wya.ctypes.data_as(dp), len(wxa), C.byref(b),
                                     C.byref(prm), C.byref(R), lo, min(S, lo + chunk))
            if rc:
                with lock:
                    state["rc"] = rc
        olib.ppo_census(cen, 1)
        with lock:
            state["census"] += np.array(cen[:], np.int64)

    ts = [threading.Thread(target=worker) for _ in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert state["rc"] == 0, state["rc"]
    return r, state["census"]


def compare_full(got, ref, chunk=16384):
    """oracle_lib.compare over the whole batch in scene chunks (bounded temporaries); returns the
    worst |dxy|, its scene, and the count of values above the tolerance."""
    S = got["winner"].shape[0]
    worst, worst_s, above = 0.0, -1, 0
    for lo in range(0, S, chunk):
        hi = min(S, lo + chunk)
        g = {k: (v[:, lo:hi] if k in ("next_x", "next_y") else v[lo:hi]) for k, v in got.items()}
        r = {k: (v[:, lo:hi] if k in ("next_x", "next_y") else v[lo:hi]) for k, v in ref.items()}
        # per-scene worst |dxy| (paths and next_x/next_y), then the strict contract on the chunk
        # (|a - b| is NaN where either is NaN or both are the same infinity: fmax skips it; the
        # NaN and infinity patterns themselves are checked exactly by compare below)
        d = np.zeros(hi - lo)
        if "paths" in r:
            e = np.abs(g["paths"] - r["paths"]).reshape(hi - lo, -1)
            d = np.fmax(d, np.fmax.reduce(e, axis=1))
            above += int(np.count_nonzero(e > oracle_lib.TOL))
            del e
        live = np.arange(g["next_x"].shape[0])[:, None] < g["n_out"][None, :]
        for k in ("next_x", "next_y"):
            e = np.abs(np.where(live, g[k], 0.0) - np.where(live, r[k], 0.0))
            d = np.fmax(d, np.fmax.reduce(e, axis=0))
            above += int(np.count_nonzero(e > oracle_lib.TOL))
        oracle_lib.compare(g, r)                  # raises on any violation of the contract
        d = np.nan_to_num(d, nan=0.0)
        i = int(np.argmax(d))
        if d[i] > worst:
            worst, worst_s = float(d[i]), lo + i
    return worst, worst_s, above


def gpu_census(config):
    """tools/limit_census.py on the census build, in a child process (one library per process)."""
    if not os.path.exists(CENSUS_LIB):
        return {"error": f"{os.path.relpath(CENSUS_LIB, REPO)} not built (make -C carnd-path-planning-project_amd census)"}
    env = dict(os.environ, PPAMD_LIB=CENSUS_LIB)
    comfort = ["--comfort"] if CONFIGS[config].get("comfort") else []
    p = subprocess.run([sys.executable, os.path.join(REPO, "tools", "limit_census.py"), "--config",
                        str(config).rstrip("c")] + comfort, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def record(config, rep):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    allr = json.load(open(OUT)) if os.path.exists(OUT) else {}
    allr[f"config{config}"] = rep
    with open(OUT, "w") as f:
        json.dump(allr, f, indent=1, sort_keys=True)


@pytest.fixture(scope="module")
def env():
    import torch
    wx, wy = oracle_lib.highway_map()
    return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy, "olib": oracle_lib.load_oracle(),
            "dev": torch.device("cuda", 0)}


@pytest.mark.parametrize("config", [5, 3, 4, "5c"])
def test_full_batch_vs_oracle(env, config):
    cfg = CONFIGS[config]
    prm = params(cfg)
    t = env["torch"]
    S = cfg["S"]
    t0 = time.time()
    scenes = ppamd.synth_device(env["m"], S, seed=0x5EED0001, first=0, device=0)
    res = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
    ppamd.evaluate(env["m"], scenes, prm, res, device=0)
    t.cuda.synchronize()
    got = ppamd.result_to_numpy(res)
    host = ppamd.scenes_to_numpy(scenes)
    del res, scenes
    t.cuda.empty_cache()
    t1 = time.time()
    with oracle_lib.quiet_stdout():
        ref, cen = oracle_full(env["olib"], env["wx"], env["wy"], host, prm)
    t2 = time.time()
    worst, worst_s, above = compare_full(got, ref)
    t3 = time.time()
    del ref, got
    g = gpu_census(config)
    rep = {"scenes": S, "candidates": S * 3 * cfg["ns"] * max(cfg["draws"], 1), "n_points": cfg["N"],
           "all_paths": cfg["paths"], "draws": cfg["draws"], "scenes_compared": S,
           "worst_dxy_m": worst, "worst_scene": worst_s, "values_above_1e-6": above,
           "oracle_decisions_941": int(cen[0]), "oracle_decisions_972": int(cen[1]),
           "oracle_near_941": int(cen[2]), "oracle_near_972": int(cen[3]),
           "gpu_census": g, "seconds": {"gpu+copy": round(t1 - t0, 1), "oracle": round(t2 - t1, 1),
                                         "compare": round(t3 - t2, 1)}}
    record(config, rep)
    print(f"\nconfig {config}: {S} scenes, every scene vs the oracle: worst |dxy| {worst:.3e} m (scene {worst_s}), "
          f"{above} values above 1e-6 m; limiter decisions :941 {cen[0]}, :972 {cen[1]}; within 1e-12 rel of "
          f"maximum_acc: {cen[2]} / {cen[3]}; GPU census {json.dumps(g)}")
    assert above == 0
    if "eval_972" in g:
        # a decision the two operation sequences take differently, if any, changed nothing the
        # contract checks (compare_full passed on every scene); it is reported, not assumed away
        assert g["eval_972"] >= 0

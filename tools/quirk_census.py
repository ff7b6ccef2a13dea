"""GPU box: strict HIP-vs-oracle census over the GPU parity tests' scene sets (emit_paths, every
candidate path). Per set: candidates whose path length or NaN pattern differs (the standstill 0/0
quirk, src/main.cpp:1025), candidates beyond 1e-6 m, and the fraction of candidate paths that are
bit-identical to the oracle's. Writes gpurun_out/census.json. Usage: python tools/quirk_census.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "carnd-path-planning-project_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
import torch  # noqa: E402
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402

wx, wy = ppamd.highway_map()
m = ppamd.Map(wx, wy)
olib = oracle_lib.load_oracle()
dev = torch.device("cuda", 0)


def todev(d):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}


def census(name, host, prm):
    S = host["ego_x"].shape[0]
    r = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    ppamd.evaluate(m, todev(host), prm, r, device=0)
    torch.cuda.synchronize()
    got = ppamd.result_to_numpy(r)
    ref = oracle_lib.oracle_eval(olib, wx, wy, host, prm, info=False)
    gp, rp = got["paths"], ref["paths"]
    nanpat = (np.isnan(gp) != np.isnan(rp)).any(axis=(1, 3))
    lendiff = got["path_len"] != ref["path_len"]
    fin = np.isfinite(gp) & np.isfinite(rp)
    err = np.where(fin, np.abs(gp - rp), 0.0).max(axis=(1, 3))
    bit = ((gp == rp) | (np.isnan(gp) & np.isnan(rp))).all(axis=(1, 3))
    out = {"scenes": S, "candidates": int(gp.shape[0] * gp.shape[2]),
           "nan_or_len_diff": int((nanpat | lendiff).sum()), "beyond_tol": int((err > 1e-6).sum()),
           "bit_identical_frac": float(bit.mean()), "max_err": float(err.max()),
           "winner_diff": int((got["winner"] != ref["winner"]).sum()),
           "status_diff": int((got["status"] != ref["status"].view(np.uint32)).sum())}
    bad = np.argwhere(nanpat | lendiff)
    out["first_bad"] = [[int(a), int(b)] for a, b in bad[:8]]
    print(name, json.dumps(out), flush=True)
    return out


res = {}
P = ppamd.default_params(emit_paths=True)
res["smoke"] = census("smoke", ppamd.scenes_to_numpy(ppamd.synth_device(m, 64, seed=1234, device=0)), P)
res["random"] = census("random", ppamd.scenes_to_numpy(ppamd.synth_device(m, 3000, seed=2024, first=10**6, device=0)), P)
import make_golden  # noqa: E402
sc, _ = make_golden.stress_pool(m, wx, wy, 3000, seed=5150)
res["stress"] = census("stress", sc, P)
P3 = ppamd.default_params(n_speeds=8, n_points=100, speed_offsets=[-6, -4, -3, -2, -1, 0, 2], emit_paths=True)
res["config3"] = census("config3", ppamd.scenes_to_numpy(ppamd.synth_device(m, 1500, seed=3, device=0)), P3)
for seed in (11, 12, 13):
    res["random_s%d" % seed] = census("random_s%d" % seed, ppamd.synth_host(m, 4000, seed=seed, first=seed * 10**7), P)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(REPO, "gpurun_out", "census.json"), "w"), indent=1)

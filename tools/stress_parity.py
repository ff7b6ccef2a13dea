"""One-off parity stress on the GPU box (not part of the suite): several seeds of synthetic scenes, of
scenes with long walks (tests/test_walks.py's generator) and of speed-edge scenes, each evaluated in
reference mode without paths (k_prep, k_cand, k_emit by rows), in all-paths mode and in comfort
mode, against the oracle under the strict contract. Prints one line per case and a summary; exit
status 1 on any mismatch.
  python3 tools/stress_parity.py [scenes per case] [seeds]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))

import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402


def main():
    import torch
    import test_walks
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    env = {"torch": torch, "m": m, "wx": wx, "wy": wy, "geo": m.geometry(),
           "olib": oracle_lib.load_oracle(), "dev": torch.device("cuda", 0)}
    worst, n = 0.0, 0
    for seed in range(seeds):
        cases = {"synthetic": ppamd.synth_host(m, S, seed=9000 + seed, first=seed * 100003),
                 "walks": test_walks.walk_scenes(env, S // 3, 7000 + seed, far=seed % 2 == 1)}
        sc = ppamd.synth_host(m, S, seed=8000 + seed, first=seed * 7)
        idx = np.arange(0, S, 7)
        sc["n_prev"][idx] = 0
        sc["ego_speed_mph"][idx] = np.array([-0.0, 5e-324, 1e-300, 3e6, 1e300, -3.0, 0.3])[np.arange(len(idx)) % 7]
        cases["speed_edges"] = sc
        for name, sc in cases.items():
            d = test_walks.to_dev(env, sc)
            for kw in ({}, {"emit_paths": True}, {"cost_mode": ppamd.COST_COMFORT}):
                prm = ppamd.default_params(**kw)
                got = test_walks.run_gpu(env, d, prm)
                ref = oracle_lib.oracle_eval(env["olib"], wx, wy, sc, prm, info=False)
                if not kw.get("emit_paths"):
                    ref = {k: v for k, v in ref.items() if k not in ("paths", "path_len")}
                e = oracle_lib.compare(got, ref)
                worst = max(worst, e)
                n += int(sc["ego_x"].shape[0])
                print(f"seed {seed} {name:12s} {str(kw):40s} scenes {sc['ego_x'].shape[0]:6d} max |dxy| {e:.3e} m",
                      flush=True)
    print(f"all cases equal the oracle: {n} scene evaluations, max |dxy| {worst:.3e} m")


if __name__ == "__main__":
    main()

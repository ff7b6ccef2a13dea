"""Debug helper (GPU box): the 100-car closed loop of tests/test_rollout.py on the GPU, the
reference's own frame code and the restatement; prints where the GPU's integer log first differs
from the reference's and, for that scene, the largest ego / plan differences of the frames before."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "carnd-path-planning-project_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402
import test_rollout  # noqa: E402


def main():
    S, F, seed = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 300, 23
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    sc, tr = test_rollout.many_car_traffic(m, S, seed)
    a, b = oracle_lib.copy_state(sc, tr), oracle_lib.copy_state(sc, tr)
    dev = torch.device("cuda", 0)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in sc.items()}
    g = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(dev) if isinstance(v, np.ndarray) else v) for k, v in tr.items()}
    prm = ppamd.default_params(n_speeds=1)
    res = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    lg = ppamd.alloc_log(F, S, 50, xp="torch", device=dev)
    ppamd.rollout(m, d, g, prm, res, F, 3, 1e5, lg)
    torch.cuda.synchronize()
    got = {k: x.cpu().numpy() for k, x in lg.items()}
    lr = oracle_lib.ref_rollout(oracle_lib.load_ref(), wx, wy, *a, F, 3, 1e5)
    lo = oracle_lib.oracle_rollout(oracle_lib.load_oracle(), wx, wy, *b, prm, F, 3, 1e5)
    for k in ("target_lane", "n_out", "n_cars", "ego_x", "plan_x"):
        print(k, "oracle==ref", np.array_equal(lo[k], lr[k]))
    bad = np.argwhere(got["target_lane"] != lr["target_lane"])
    print("target_lane mismatches (frame, scene):", bad[:10].tolist())
    for f, s in bad[:3]:
        lo_f = max(0, f - 8)
        for q in range(lo_f, f + 1):
            de = max(abs(got["ego_x"][q, s] - lr["ego_x"][q, s]), abs(got["ego_y"][q, s] - lr["ego_y"][q, s]))
            n = int(lr["n_out"][q, s])
            dp = np.abs(got["plan_x"][q, :n, s] - lr["plan_x"][q, :n, s]).max() if n else 0.0
            print(f"  scene {s} frame {q}: tl gpu {got['target_lane'][q, s]} ref {lr['target_lane'][q, s]} "
                  f"oracle {lo['target_lane'][q, s]}  |d ego| {de:.3e}  |d plan| {dp:.3e}  status {got['status'][q, s]:#x}")


if __name__ == "__main__":
    main()

"""Debug helper (GPU box): evaluate synthetic scenes on the GPU and with the oracle, dump the
scenes whose integer outputs or paths disagree into gpurun_out/mismatch.npz."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "carnd-path-planning-project_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402

wx, wy = ppamd.highway_map()
m = ppamd.Map(wx, wy)
S = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
prm = ppamd.default_params(emit_paths=True)
sc = ppamd.synth_device(m, S, seed=2024, first=10**6, device=0)
r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
ppamd.evaluate(m, sc, prm, r, device=0)
torch.cuda.synchronize()
got = ppamd.result_to_numpy(r)
host = ppamd.scenes_to_numpy(sc)
ref = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, host, prm, info=True)
bad_len = np.nonzero((got["path_len"] != ref["path_len"]).any(1))[0]
d = np.abs(np.nan_to_num(got["paths"], nan=1e9) - np.nan_to_num(ref["paths"], nan=1e9)).reshape(S, -1).max(1)
bad_xy = np.nonzero(d > 1e-6)[0]
print("path_len mismatching scenes:", len(bad_len), bad_len[:20])
print("xy mismatching scenes:", len(bad_xy), bad_xy[:20])
for s in bad_len[:5]:
    c = np.nonzero(got["path_len"][s] != ref["path_len"][s])[0]
    print("scene", s, "cands", c, "gpu", got["path_len"][s][c], "oracle", ref["path_len"][s][c],
          "status gpu %x oracle %x" % (got["status"][s], ref["status"][s]))
bad = np.union1d(bad_len, bad_xy)
np.savez(os.path.join(REPO, "gpurun_out", "mismatch.npz"), idx=bad,
         **{"scene_" + k: v[..., bad] for k, v in host.items()},
         gpu_paths=got["paths"][bad], gpu_len=got["path_len"][bad], gpu_cost=got["cost"][bad],
         gpu_status=got["status"][bad])

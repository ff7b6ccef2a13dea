"""K0 debugging: the one-lane K1 with k_sort_cars (G = 1) against the grouped K1 (G = 2, no K0)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
import torch, ppamd
dev = torch.device("cuda", 0)
m = ppamd.Map(*ppamd.highway_map())
for emit in (False, True):
    S = 70000
    prm = ppamd.default_params(emit_paths=emit)
    sc = ppamd.synth_device(m, S, seed=0x5EED0003, device=0)
    out = {}
    for g in (1, 2):
        r = ppamd.alloc_result(S, prm, xp="torch", device=dev, info=True)
        with ppamd.debug(ppamd.DBG_PREP_GROUP, g):
            ppamd.evaluate(m, sc, prm, r, device=0)
        torch.cuda.synchronize()
        out[g] = ppamd.result_to_numpy(r)
    a, b = out[1], out[2]
    bad = np.nonzero((a["cost"].view(np.uint64) != b["cost"].view(np.uint64)).any(1))[0]
    print("emit", emit, "scenes with cost differences:", len(bad), bad[:10])
    for k in a["info"].dtype.names:
        x, y = a["info"][k], b["info"][k]
        d = np.nonzero((x != y) & ~(np.isnan(x) & np.isnan(y)) if x.dtype.kind == 'f' else (x != y))[0] if x.ndim == 1 else []
        if len(d): print("  info", k, len(d), d[:5], x[d[:3]], y[d[:3]])
    if len(bad):
        s = bad[0]
        print("  scene", s, "cost K0", a["cost"][s][:6], "grouped", b["cost"][s][:6])
        h = ppamd.scenes_to_numpy(sc)
        print("  n_cars", h["n_cars"][s], "n_prev", h["n_prev"][s], "ids", h["car_id"][:, s])

"""Debug helper (GPU box): the speed-edge scenes of tests/test_gpu_parity.py
(test_speed_range_edges_vs_oracle), printing every scene whose status word differs from the
oracle's with the differing bits, the telemetry speed and the in-lane car's velocity."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "carnd-path-planning-project_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
import oracle_lib  # noqa: E402
from oracle_lib import ppamd  # noqa: E402

wx, wy = oracle_lib.highway_map()
m = ppamd.Map(wx, wy)
S = 1200
sc = ppamd.synth_host(m, S, seed=909, first=31337)
speeds = [-0.0, 0.0, 5e-324, 1e-310, 1e-300, 1e-40, 1e-18, 2.237e-17, 1e-12, 1e-6, 0.3,
          49.66, 3e6, 1e300, -3.0, -1e-300, 2.237 * 22.2]
vels = [0.0, -0.0, 5e-324, 1e-300, 1e-25, 1e-9, 3.0]
p9x, p9y = sc["prev_x"][9], sc["prev_y"][9]
hx, hy = p9x - sc["prev_x"][8], p9y - sc["prev_y"][8]
nrm = np.maximum(np.hypot(hx, hy), 1e-12)
for s in range(S):
    if s % 3 != 2:
        sc["n_prev"][s] = 0
        sc["ego_speed_mph"][s] = speeds[s % len(speeds)]
    if s % 2 == 0:
        sc["car_x"][0, s] = p9x[s] + hx[s] / nrm[s] * 20.0
        sc["car_y"][0, s] = p9y[s] + hy[s] / nrm[s] * 20.0
        v = vels[(s // 2) % len(vels)]
        sc["car_vx"][0, s] = v
        sc["car_vy"][0, s] = v
names = {v: k for k, v in ppamd.STATUS_BITS.items()}
for emit in (True, False):
    prm = ppamd.default_params(emit_paths=emit)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in sc.items()}
    r = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
    ppamd.evaluate(m, dev, prm, r, device=0)
    torch.cuda.synchronize()
    got = ppamd.result_to_numpy(r)
    ref = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, sc,
                                 ppamd.default_params(emit_paths=True), info=False)
    rs = ref["status"].view(np.uint32)
    bad = np.nonzero(got["status"] != rs)[0]
    print(f"emit={emit}: {len(bad)} scenes with differing status; winners differ at "
          f"{np.count_nonzero(got['winner'] != ref['winner'])}")
    for s in bad[:40]:
        x = int(got["status"][s] ^ rs[s])
        bits = [names.get(1 << b, str(b)) for b in range(32) if x >> b & 1]
        print(f"  s={s} gpu={got['status'][s]:#x} ref={rs[s]:#x} diff={bits} n_prev={sc['n_prev'][s]} "
              f"speed={sc['ego_speed_mph'][s]!r} car0 v={sc['car_vx'][0, s]!r} "
              f"win gpu {got['winner'][s]} ref {ref['winner'][s]} n_out {got['n_out'][s]}/{ref['n_out'][s]}")

"""PCIe copy ceilings for the host-buffer mode (bench.py host_pipeline): pinned host
<-> device copies of config 5's per-step bytes (1.33 GB in, 1.95 GB out), each direction alone and
both at once on two streams, as one copy per direction or in chunks. GPU box:
  python3 tools/pcie_probe.py [--chunks 8] [--reps 5]"""
import argparse
import json
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--chunks", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--h2d-gb", type=float, default=1.3338)
ap.add_argument("--d2h-gb", type=float, default=1.9545)
a = ap.parse_args()
dev = torch.device("cuda", 0)
nin, nout = int(a.h2d_gb * 1e9) // 8, int(a.d2h_gb * 1e9) // 8
h_in = torch.empty(nin, dtype=torch.float64).pin_memory()
h_out = torch.empty(nout, dtype=torch.float64).pin_memory()
d_in = torch.empty(nin, dtype=torch.float64, device=dev)
d_out = torch.zeros(nout, dtype=torch.float64, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def parts(n, k):
    return [(i * n // k, (i + 1) * n // k) for i in range(k)]


def run(h2d, d2h, k):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if h2d:
        with torch.cuda.stream(s1):
            for lo, hi in parts(nin, k):
                d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
    if d2h:
        with torch.cuda.stream(s2):
            for lo, hi in parts(nout, k):
                h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3


res = {}
for name, h2d, d2h in (("h2d", 1, 0), ("d2h", 0, 1), ("both", 1, 1)):
    for k in (1, a.chunks):
        run(h2d, d2h, k)
        t = sorted(run(h2d, d2h, k) for _ in range(a.reps))
        gb = (nin * 8 if h2d else 0) + (nout * 8 if d2h else 0)
        res[f"{name}_x{k}"] = {"ms_median": round(t[len(t) // 2], 2), "ms_min": round(t[0], 2),
                               "GB_per_s": round(gb / 1e9 / (t[len(t) // 2] / 1e3), 1)}
        print(name, k, res[f"{name}_x{k}"], flush=True)
print(json.dumps(res))

"""Probe (GPU box): whole config-5 batches with 1, 2 or 3 of them in flight on separate HIP streams
(one result buffer and one pp_eval workspace per stream), steps alternating over the streams.
Prints ms per batch for each depth."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "carnd-path-planning-project_amd"))
import torch
import ppamd

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2097152
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
wx, wy = ppamd.highway_map()
prm = ppamd.default_params()
m = ppamd.Map(wx, wy)
m.reserve(0, S)
scenes = ppamd.synth_device(m, S, device=0, stream=torch.cuda.current_stream().cuda_stream)
for depth in (1, 2, 3, 1, 2):
    streams = [torch.cuda.Stream(dev) for _ in range(depth)]
    res = [ppamd.alloc_result(S, prm, xp="torch", device=dev) for _ in range(depth)]
    torch.cuda.synchronize()

    def run(k):
        for i in range(k):
            ppamd.evaluate(m, scenes, prm, res[i % depth], device=0, stream=streams[i % depth].cuda_stream)
    run(2 * depth)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(30)
    torch.cuda.synchronize()
    print(f"depth {depth}: {(time.perf_counter() - t0) / 30 * 1e3:.3f} ms/batch", flush=True)
    del res

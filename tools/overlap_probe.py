"""Probe (GPU box): does splitting the config-5 batch into chunks on two HIP streams (k_prep / k_emit
of one chunk overlapping k_cand of another) shorten the step? Uses one Map (own workspace) per
chunk so no kernel change is needed. Prints ms per full batch for 1 stream vs 2 streams."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "carnd-path-planning-project_amd"))
import torch
import ppamd

S = 2097152
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
wx, wy = ppamd.highway_map()
prm = ppamd.default_params()
for nch in (1, 2, 4, 8):
    Sc = S // nch
    maps, scenes, res = [], [], []
    for c in range(nch):
        m = ppamd.Map(wx, wy)
        m.reserve(0, Sc)
        maps.append(m)
        scenes.append(ppamd.synth_device(m, Sc, first=c * Sc, device=0, stream=torch.cuda.current_stream().cuda_stream))
        res.append(ppamd.alloc_result(Sc, prm, xp="torch", device=dev))
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    torch.cuda.synchronize()
    for mode in ("1stream", "2streams"):
        def step():
            for c in range(nch):
                st = streams[0] if mode == "1stream" else streams[c % 2]
                ppamd.evaluate(maps[c], scenes[c], prm, res[c], device=0, stream=st.cuda_stream)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            step()
        torch.cuda.synchronize()
        print(f"chunks {nch} {mode}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms/batch", flush=True)
    del maps, scenes, res

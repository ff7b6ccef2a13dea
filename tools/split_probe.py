"""Step time of one shard-sized batch (default 262,144 scenes, BASELINE config 5's share at N = 8)
with the split on and off, without pp_timing's events, with K2's only (timing 2, the bench's timed
region) and with every kernel's (timing 1): the events cost stream time. GPU box: python3 tools/split_probe.py [S] [reps] [steps]."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
import torch  # noqa: E402
import ppamd  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params()
    m.reserve(0, S)
    sp = torch.cuda.current_stream(dev).cuda_stream
    sc = ppamd.synth_device(m, S, seed=0x5EED0001, first=0, device=0, stream=sp)
    res = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    for _ in range(reps):
        for split in (ppamd.SPLIT_ON, ppamd.SPLIT_OFF):
            for timing in (0, ppamd.TIMING_K2, ppamd.TIMING_ALL):
                with ppamd.debug(ppamd.DBG_SPLIT, split):
                    for _ in range(3):
                        ppamd.evaluate(m, sc, prm, res, device=0, stream=sp)
                    torch.cuda.synchronize(dev)
                    m.timing(0, timing)
                    t = time.perf_counter()
                    for _ in range(steps):
                        ppamd.evaluate(m, sc, prm, res, device=0, stream=sp)
                    torch.cuda.synchronize(dev)
                    ms = (time.perf_counter() - t) / steps * 1e3
                    k = m.read_timing(0) if timing else None
                    m.timing(0, False)
                print(f"split {'on ' if split == ppamd.SPLIT_ON else 'off'} timing {int(timing)}: {ms:.4f} ms/step",
                      "" if k is None else f"kernels {[round(a / max(b, 1), 4) for a, b in zip(*k)]}", flush=True)


if __name__ == "__main__":
    main()

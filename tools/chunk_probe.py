"""Round 6: does BASELINE config 5's batch (2,097,152 scenes) run faster as
sequential chunks? Step time, no timing events, same process and box, alternating:
  full    one pp_eval of the whole batch (the library's policy: one stream)
  split   one pp_eval with the split forced on (PP_DBG_SPLIT 1)
  cK      K sequential pp_eval calls of S / K scenes each (each under the library's policy: 1 M and
          512 k scenes run as 3 parts on 3 streams), the same scenes as the full batch
GPU box: python3 tools/chunk_probe.py [reps] [steps]."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
import torch  # noqa: E402
import ppamd  # noqa: E402

S = 2097152


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params()
    m.reserve(0, S)
    sp = torch.cuda.current_stream(dev).cuda_stream
    full = (ppamd.synth_device(m, S, seed=0x5EED0001, first=0, device=0, stream=sp),
            ppamd.alloc_result(S, prm, xp="torch", device=dev))
    chunks = {}
    for K in (2, 4):
        n = S // K
        chunks[K] = [(ppamd.synth_device(m, n, seed=0x5EED0001, first=k * n, device=0, stream=sp),
                      ppamd.alloc_result(n, prm, xp="torch", device=dev)) for k in range(K)]
    torch.cuda.synchronize(dev)

    def run(name):
        if name == "full":
            ppamd.evaluate(m, full[0], prm, full[1], device=0, stream=sp)
        elif name == "split":
            with ppamd.debug(ppamd.DBG_SPLIT, ppamd.SPLIT_ON):
                ppamd.evaluate(m, full[0], prm, full[1], device=0, stream=sp)
        else:
            for sc, res in chunks[int(name[1:])]:
                ppamd.evaluate(m, sc, prm, res, device=0, stream=sp)

    for r in range(reps):
        for name in ("full", "split", "c2", "c4"):
            for _ in range(3):
                run(name)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(steps):
                run(name)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t) / steps * 1e3
            print(f"rep {r} {name:5s} {ms:.4f} ms/step", flush=True)
    # the chunks produce the full batch's results (same scenes, same kernels): bit for bit
    run("full")
    run("c2")
    torch.cuda.synchronize(dev)
    n = S // 2
    for k, (_, res) in enumerate(chunks[2]):
        for key in ("winner", "n_out", "status"):
            assert torch.equal(res[key], full[1][key][k * n:(k + 1) * n]), key
        for key in ("next_x", "next_y"):
            assert torch.equal(res[key].view(torch.int64), full[1][key][:, k * n:(k + 1) * n].view(torch.int64)), key
        assert torch.equal(res["cost"].view(torch.int64), full[1]["cost"][k * n:(k + 1) * n].view(torch.int64))
    print("c2 == full bit for bit")


if __name__ == "__main__":
    main()

"""bench.py — candidate trajectories/s of the MI355X evaluator (BASELINE.json metric).

A step = one pp_eval over one resident batch of synthetic scenes (inputs already in HBM): K1 scene
prep + K2 candidate evaluation (3 lanes x n_speeds, 50-point horizon, spline + limiter + cost)
+ the per-scene winner path. Default workload = BASELINE config 5: 2,097,152 scenes x 15
candidates IN TOTAL, sharded over the N GPUs (strong scaling: rank r evaluates the contiguous
global scenes [r S/N, (r+1) S/N) of one seeded synthetic stream). No collective on the data path:
the ranks meet only in the timing barrier and the max over ranks, both over gloo on the host.
For N > 1 the line also carries a weak-scaling measurement (2,097,152 scenes per GPU).

Run: python bench.py [--gpus N --steps K --warmup W]. Under torch.distributed.run (WORLD_SIZE set)
each process is one rank; without it, --gpus N > 1 starts N rank processes itself (the parent
never touches the GPU) and exits with their status.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "carnd-path-planning-project_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
SCENE_BYTES = 4 * 8 + 20 * 8 + 3 * 4 + 12 * (4 + 4 * 8)   # SoA scene record (include/pp.h): 636 B
CONFIG5_SCENES = 2_097_152


def algorithmic_bytes_per_candidate(C_, N, emit_paths):
    """scene record read once per scene, winner path + n_out/winner written once
    per scene, one f64 cost per candidate; all-paths mode writes every candidate's N points."""
    if emit_paths:
        return (SCENE_BYTES + 8) / C_ + 8 + 16 * N + 4
    return (SCENE_BYTES + 8 + 16 * N) / C_ + 8


def shard(rank, world, total=None, per_rank=None):
    """Scene range (first, count) of `rank`. Strong scaling (total given): contiguous balanced
    shards of `total` global scenes; weak scaling (per_rank given): [rank * per_rank, ...).
    Scenes depend only on (seed, global index), so any layout evaluates the same scenes."""
    if total is not None:
        lo = rank * total // world
        hi = (rank + 1) * total // world
        return lo, hi - lo
    return rank * per_rank, per_rank


def max_over_ranks(elapsed, dist, device=None):
    """The job's time is the slowest rank's: MAX all-reduce of a host tensor over the gloo group."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_envs(n, port, base=None):
    """Environments of the n rank processes the launcher starts (torch.distributed.run's names)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        envs.append(e)
    return envs


def launch(n, argv):
    """Start n rank processes of this script (the parent has not touched the GPU) and wait for them;
    rank 0 prints the JSON line. Returns the worst exit status."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e)
             for e in rank_envs(n, free_port())]
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def load_valu_peak():
    """Measured FP64 VALU issue rate (tools/valu_peak.hip on the MI355X, profiles/r01_valu_peak.json)."""
    p = os.path.join(REPO, "profiles", "r01_valu_peak.json")
    try:
        j = json.load(open(p))
        return j["v_fma_f64"]["wave_instr_per_s"], j["v_add_f64"]["wave_instr_per_s"]
    except Exception:
        return None, None


def load_pmc_all():
    """The committed rocprofv3 PMC summary (profiles/pmc_summary.json): per launch-shape tag."""
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        return json.load(open(p))
    except Exception:
        return {}


def load_rocprof_all():
    """The committed rocprofv3 kernel-trace summary (profiles/rocprof_summary.json, written by
    tools/rocprof_summarize.py): per launch-shape tag, the profiler's average K2 launch duration."""
    p = os.path.join(REPO, "profiles", "rocprof_summary.json")
    try:
        return json.load(open(p))
    except Exception:
        return {}


def stamped(entry, sha):
    """A profile summary entry (pmc_summary.json / rocprof_summary.json) applies to this run only if
    it was measured on the same library build: its lib_sha256 equals the loaded library's."""
    return bool(entry) and entry.get("lib_sha256") == sha


def profile_entries(pmc, rp, sha):
    """(pmc, rp, stamp): the PMC and kernel-trace entries of this launch shape kept only when their
    library stamp matches the loaded library (else None: their counts describe another binary), and
    a record of which were dropped."""
    stamp = {"lib_sha256": sha,
             "pmc": None if not pmc else ("match" if stamped(pmc, sha) else "stale: " + str(pmc.get("lib_sha256"))),
             "rocprof": None if not rp else ("match" if stamped(rp, sha) else "stale: " + str(rp.get("lib_sha256")))}
    return (pmc if stamped(pmc, sha) else None), (rp if stamped(rp, sha) else None), stamp


def shard_projection(t_full, t_shards):
    """Projected strong-scaling speed-ups of config 5 from same-process shard timings (a PROJECTION,
    not a multi-GPU measurement): N GPUs each evaluate one 1/N shard (no collective), so the job
    takes the shard's time. The one-GPU time it is compared with is the batch under its best
    single-GPU policy (like with like): one pp_eval call of the whole batch, or
    the N shards' calls one after another on the one GPU (N x t(shard)); so the speed-up is
    min(t(full), N t(shard)) / t(shard) <= N. speedup_vs_one_call keeps t(full) / t(shard)."""
    out = {}
    for n, t in sorted(t_shards.items()):
        t1 = min(t_full, n * t)
        out[str(n)] = {"speedup": t1 / t, "efficiency": t1 / t / n, "shard_ms_per_step": t * 1e3,
                       "one_gpu_ms_per_step": t1 * 1e3,
                       "one_gpu_policy": "one call" if t_full <= n * t else f"{n} shard calls in sequence",
                       "speedup_vs_one_call": t_full / t}
    return out


def pmc_tag(S, Cn, N, emit_paths, D, comfort=False):
    return (f"k_cand_S{S}_C{Cn}_N{N}" + ("_paths" if emit_paths else "") + (f"_D{D}" if D > 1 else "")
            + ("_comfort" if comfort else ""))


def pmc_for(pmc_all, S, Cn, N, emit_paths, D, comfort=False):
    """The PMC entry of this launch shape: the exact tag, else the largest profiled launch with the
    same candidates per scene, horizon, paths mode and draws (counter bytes and instructions per
    candidate carry over between batch sizes of one shape). Entries must state their launch size
    (candidates_per_launch): a counter total is meaningless without it."""
    exact = pmc_all.get(pmc_tag(S, Cn, N, emit_paths, D, comfort))
    cands = [exact] if exact else [
        e for e in pmc_all.values()
        if (e.get("candidates_per_scene"), e.get("n_points"), e.get("emit_paths"), e.get("draws", 1),
            bool(e.get("comfort"))) == (Cn, N, bool(emit_paths), D, bool(comfort))]
    if not cands:
        return None
    e = max(cands, key=lambda e: e.get("candidates_per_launch") or 0)
    if not e.get("candidates_per_launch"):
        raise ValueError(f"profiles/pmc_summary.json entry without candidates_per_launch: {e.get('source')}")
    return e


def workload_name(S, Cn, n_speeds, N, emit_paths, D, rollout):
    """Which BASELINE.json config a run measures (configs[1..4] = configs 2..5)."""
    if rollout:
        return "closed-loop rollout (SURVEY.md §8(f) row 1)"
    if D > 1 and n_speeds == 1 and N == 50:
        return "BASELINE config 4"
    if emit_paths and n_speeds == 8 and N == 100:
        return "BASELINE config 3"
    if S == 4096 and n_speeds == 5 and N == 50 and not emit_paths and D == 1:
        return "BASELINE config 2"
    if n_speeds == 5 and N == 50 and not emit_paths and D == 1:
        return "BASELINE config 5"
    return "custom workload"


def workload_scope(wname, S, total, world, scaling):
    """How the run's scenes relate to the named workload: the whole config-5 batch sharded over the
    ranks, one rank-sized shard of it measured alone (e.g. 262,144 scenes = its share at N = 8), or
    a fixed batch per GPU."""
    if scaling == "weak":
        return f" ({S} per GPU)"
    if wname == "BASELINE config 5" and total != CONFIG5_SCENES:
        return (f" (one shard of the {CONFIG5_SCENES}-scene batch: its share at N = {CONFIG5_SCENES // total}"
                if CONFIG5_SCENES % total == 0 else " (a partial batch") + f", measured on {world} GPU(s))"
    return f" sharded over {world} GPUs"


def roofline_fields(pmc, cands_launch, bpc, k_ms):
    """traffic (dominant kernel) and traffic_pipeline (every kernel of a step) per launch of this
    run, from the PMC entry's bytes per candidate."""
    if not pmc:
        return None, None
    pc = pmc["candidates_per_launch"]
    traffic = pmc["hbm_bytes_per_launch"] / pc * cands_launch
    pipe = pmc["pipeline_bytes_per_step"] / pc * cands_launch if pmc.get("pipeline_bytes_per_step") else None
    return traffic, pipe


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scenes", type=int, default=CONFIG5_SCENES,
                    help="total scenes (strong scaling) or scenes per GPU (--scaling weak)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong")
    ap.add_argument("--n-speeds", type=int, default=5)
    ap.add_argument("--n-points", type=int, default=50)
    ap.add_argument("--emit-paths", action="store_true", help="write every candidate path (config 3)")
    ap.add_argument("--comfort", action="store_true", help="comfort cost mode (data-dependent argmin)")
    ap.add_argument("--draws", type=int, default=0,
                    help="Monte-Carlo sensor-noise draws per scene (config 4: --scenes 16384 --draws 64 --n-speeds 1)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="closed-loop mode: one step = this many pp_rollout frames (plan + simulator)")
    ap.add_argument("--sensor-range", type=float, default=300.0)
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline time budget per leg")
    ap.add_argument("--cpu-threads", type=int, default=0, help="all-core leg threads (0: the host's CPU share)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the extra weak-scaling measurement")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) side measurement")
    ap.add_argument("--pcie-chunks", type=int, default=8,
                    help="chunks of the host-buffer pipeline (H2D / evaluate / D2H overlapped across chunks)")
    ap.add_argument("--debug", action="append", default=[], metavar="KEY=VALUE",
                    help="library debug switch for A/B runs (include/pp.h PP_DBG_*): prep_group=G, "
                         "prep_waves=3|4, shape=1|2|3, split=1|2, sort_cars=1|2; recorded in config.debug, which marks the line not reportable")
    ap.add_argument("--no-comfort", action="store_true",
                    help="skip the comfort-mode (data-dependent argmin) side measurement of config 5 (1 GPU)")
    ap.add_argument("--no-shard-projection", action="store_true",
                    help="skip timing config 5's 2-, 4- and 8-GPU shards after the headline (1 GPU, config 5)")
    ap.add_argument("--cpu-ranks", action="store_true",
                    help="launcher rehearsal without a GPU: every rank evaluates its shard with the CPU oracle")
    return ap.parse_args(argv)


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        share = min(share, int(omp))
    return model, os.cpu_count(), max(1, min(share, 64))


def cpu_baseline(scenes_host_fn, S, prm, budget_s, threads):
    """The reference's own planning code (oracle/_ref, compiled from the reference's sources) if it
    was built, else the C restatement (oracle/liboracle.so): one host core, then `threads` cores
    (std::thread-like: Python threads around the GIL-free ctypes call, static chunk partition),
    each leg over a bounded sample of the same synthetic batch."""
    import threading
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    import ppamd
    wx, wy = ppamd.highway_map()
    rlib = oracle_lib.load_ref() if prm.n_points == 50 and not prm.emit_paths and prm.n_draws <= 1 else None
    olib = None if rlib else oracle_lib.load_oracle()
    offs = [prm.speed_offsets[i] for i in range(prm.n_speeds - 1)]
    chunk = 1024
    cand_per_scene = 3 * prm.n_speeds * max(prm.n_draws, 1)

    def run_chunk(host):
        if rlib:
            oracle_lib.ref_eval(rlib, wx, wy, host, prm.n_speeds, offs, with_frame=False)
        else:
            oracle_lib.oracle_eval(olib, wx, wy, host, prm, info=False)

    def leg(nthreads):
        """Scenes done / wall time with nthreads workers pulling chunks until the budget ends."""
        lock = threading.Lock()
        state = {"next": 0, "done": 0}
        t0 = time.perf_counter()

        def worker():
            while True:
                with lock:
                    if time.perf_counter() - t0 > budget_s or state["next"] >= S:
                        return
                    start = state["next"]
                    state["next"] += chunk
                host = scenes_host_fn(start, min(chunk, S - start))
                run_chunk(host)
                with lock:
                    state["done"] += host["ego_x"].shape[0]

        ts = [threading.Thread(target=worker) for _ in range(nthreads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return state["done"], time.perf_counter() - t0

    # the reference's printf warnings ("detected collision", "spline input error") go to fd 1: keep
    # them out of the bench's one-line JSON stdout
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    try:
        d1, t1 = leg(1)
        dn, tn = leg(threads) if threads > 1 else (d1, t1)
    finally:
        import ctypes
        ctypes.CDLL(None).fflush(None)           # C stdio buffers drain into /dev/null too
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    model, nproc, _ = host_cpu()
    src = "reference src/main.cpp classes built by oracle/Makefile" if rlib else "C restatement oracle/pp_oracle.c"
    return {"value": dn * cand_per_scene / tn, "unit": "candidate trajectories/s", "cores": threads,
            "kind": "reference" if rlib else "port",
            "value_1core": d1 * cand_per_scene / t1, "nproc": nproc, "cpu_model": model,
            "sample": f"{dn} scenes x {cand_per_scene} candidates of the same synthetic batch on {threads} "
                      f"threads ({tn:.1f} s), and {d1} scenes on 1 thread ({t1:.1f} s); {src}"}


def chunk_bounds(S, chunks):
    """Contiguous balanced scene ranges [lo, hi) of the host-buffer pipeline's chunks."""
    k = max(1, min(chunks, S))
    return [(i * S // k, (i + 1) * S // k) for i in range(k)]


OUT_FIELDS = ("winner", "n_out", "next_x", "next_y", "cost", "status")


def host_pipeline(m, scenes, prm, device, chunks, steps, warmup):
    """PCIe-inclusive rate: the batch starts and ends in pinned host memory, as a
    server handing pp_eval host buffers would see it. The batch is cut into `chunks` scene ranges;
    chunk k's H2D copy, its pp_eval and its D2H copy (winner, n_out, next_x/y, costs, status) run
    on three streams, double-buffered, so the copies of one chunk overlap the evaluation of the
    next. Returns scenes/s-derived figures for the timed steps (the caller scales by candidates)."""
    import torch
    import ppamd
    dev = torch.device("cuda", device)
    S = int(scenes["ego_x"].shape[0])
    bounds = chunk_bounds(S, chunks)
    # pinned host copies of every chunk (chunk-shaped SoA, as a host caller would hold them)
    h_sc = [{k: v[..., lo:hi].contiguous().cpu().pin_memory() for k, v in scenes.items()} for lo, hi in bounds]
    h_res = [{k: v.pin_memory() for k, v in ppamd.alloc_result(hi - lo, prm, xp="torch", device="cpu").items()
              if k in OUT_FIELDS} for lo, hi in bounds]
    cmax = max(hi - lo for lo, hi in bounds)
    # double buffers as flat storage sized for the largest chunk; chunk k uses compact views of
    # its own shape over the front of them (the SoA layout [row * n + s] needs n as the stride)
    d_sc = [{k: torch.empty(v[..., :1].numel() * cmax, dtype=v.dtype, device=dev) for k, v in scenes.items()}
            for _ in range(2)]
    r_tmpl = {k: v for k, v in ppamd.alloc_result(cmax, prm, xp="torch", device="cpu").items()}
    d_res = [{k: torch.empty(v.numel(), dtype=v.dtype, device=dev) for k, v in r_tmpl.items()} for _ in range(2)]
    s_h2d, s_cmp, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))
    m.reserve(device, cmax)
    h2d_bytes = sum(t.numel() * t.element_size() for c in h_sc for t in c.values())
    d2h_bytes = sum(t.numel() * t.element_size() for c in h_res for t in c.values())

    def compact(flat, shape):
        n = 1
        for x in shape:
            n *= x
        return flat[:n].view(shape)

    def view(d, k):
        return {f: compact(t, h_sc[k][f].shape) for f, t in d.items()}

    def rview(d, k, n):
        shapes = {f: (v.shape[0], n) if f in ("next_x", "next_y") else (n,) + tuple(v.shape[1:])
                  for f, v in r_tmpl.items()}
        return {f: compact(t, shapes[f]) for f, t in d.items()}

    def one_step():
        ev_cmp = [None] * len(bounds)
        ev_d2h = [None] * len(bounds)
        for k, (lo, hi) in enumerate(bounds):
            n, b = hi - lo, k % 2
            sc_k, rs_k = view(d_sc[b], k), rview(d_res[b], k, n)
            with torch.cuda.stream(s_h2d):
                if k >= 2:
                    s_h2d.wait_event(ev_cmp[k - 2])          # chunk k-2 is done with d_sc[b]
                for f, t in sc_k.items():
                    t.copy_(h_sc[k][f], non_blocking=True)
                e_in = torch.cuda.Event()
                e_in.record(s_h2d)
            s_cmp.wait_event(e_in)
            if k >= 2:
                s_cmp.wait_event(ev_d2h[k - 2])              # chunk k-2's results have left d_res[b]
            ppamd.evaluate(m, sc_k, prm, rs_k, device=device, stream=s_cmp.cuda_stream)
            ev_cmp[k] = torch.cuda.Event()
            ev_cmp[k].record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(ev_cmp[k])
                for f in OUT_FIELDS:
                    h_res[k][f].copy_(rs_k[f], non_blocking=True)
                ev_d2h[k] = torch.cuda.Event()
                ev_d2h[k].record(s_d2h)

    for _ in range(warmup):
        one_step()
    torch.cuda.synchronize(dev)
    # each step host buffer to host buffer, timed on its own (the copy engines' rate varies from step
    # to step on the box): the median step is reported, the mean and the fastest beside it
    per = []
    for _ in range(steps):
        t0 = time.perf_counter()
        one_step()
        torch.cuda.synchronize(dev)
        per.append(time.perf_counter() - t0)
    el = float(np.median(per)) * steps
    # the host-side outputs, reassembled in scene order before copy_rate below reuses the buffers
    # (tests compare them with the resident path)
    outs = {f: torch.cat([h[f] for h in h_res], dim=1 if f in ("next_x", "next_y") else 0) for f in OUT_FIELDS}

    def copy_rate(h2d):
        """One direction alone: every chunk's copies on one stream, GB/s."""
        s = s_h2d if h2d else s_d2h
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        with torch.cuda.stream(s):
            for k, (lo, hi) in enumerate(bounds):
                if h2d:
                    for f, d in view(d_sc[k % 2], k).items():
                        d.copy_(h_sc[k][f], non_blocking=True)
                else:
                    for f, d in rview(d_res[k % 2], k, hi - lo).items():
                        if f in OUT_FIELDS:
                            h_res[k][f].copy_(d, non_blocking=True)
        torch.cuda.synchronize(dev)
        return (h2d_bytes if h2d else d2h_bytes) / (time.perf_counter() - t) / 1e9

    stats = {"scenes_per_s": S * steps / el, "ms_per_step": el / steps * 1e3, "chunks": len(bounds),
             "ms_per_step_mean": float(np.mean(per)) * 1e3, "ms_per_step_min": float(np.min(per)) * 1e3,
             "h2d_only_gb_per_s": copy_rate(True), "d2h_only_gb_per_s": copy_rate(False),
             "h2d_bytes_per_step": h2d_bytes, "d2h_bytes_per_step": d2h_bytes,
             "pcie_gb_per_s": (h2d_bytes + d2h_bytes) * steps / el / 1e9}
    return stats, outs


def run_cpu_ranks(a, rank, world, dist):
    """--cpu-ranks: the launcher, sharding and timing protocol rehearsed without a GPU (CPU oracle)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    import ppamd
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    olib = oracle_lib.load_oracle()
    prm = ppamd.default_params(n_speeds=a.n_speeds)
    first, n = shard(rank, world, total=a.scenes) if a.scaling == "strong" else shard(rank, world, per_rank=a.scenes)
    sc = ppamd.synth_host(m, n, seed=a.seed, first=first)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = oracle_lib.oracle_eval(olib, wx, wy, sc, prm, info=False)
    if dist:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist)
    digest = float(np.nansum(r["cost"]))
    digests = [digest]
    shards = [(first, n)]
    if dist:
        digests = [None] * world
        shards = [None] * world
        dist.all_gather_object(digests, digest)
        dist.all_gather_object(shards, (first, n))
    total = sum(c for _, c in shards)
    return {"metric": "candidate trajectories/sec (CPU rehearsal of the rank launcher)", "value":
            total * 3 * a.n_speeds * a.steps / elapsed, "n_gpus": world, "steps": a.steps,
            "scaling": a.scaling, "shards": shards, "cost_digests": digests, "ms_per_step": elapsed / a.steps * 1e3}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return launch(a.gpus, argv)
    world = int(env_world or "1")
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    if a.cpu_ranks:
        out = run_cpu_ranks(a, rank, world, dist)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return 0

    import torch
    import ppamd
    keys = {"prep_group": ppamd.DBG_PREP_GROUP, "prep_waves": ppamd.DBG_PREP_WAVES, "shape": ppamd.DBG_SHAPE,
            "split": ppamd.DBG_SPLIT, "sort_cars": ppamd.DBG_SORT_CARS}
    for kv in a.debug:
        k, _, v = kv.partition("=")
        ppamd.debug_set(keys[k], int(v))
    # one GPU per local rank; more local ranks than GPUs share them round-robin (a rehearsal of the
    # N-rank path on a smaller box: a per-GPU timing is then not a scaling figure)
    ngpu = torch.cuda.device_count()
    local = local % ngpu if ngpu else local
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params(n_speeds=a.n_speeds, n_points=a.n_points,
                               cost_mode=ppamd.COST_COMFORT if a.comfort else ppamd.COST_REFERENCE,
                               emit_paths=a.emit_paths, n_draws=a.draws, noise_first_scene=0,
                               speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if a.n_speeds == 8 else None)
    D = max(a.draws, 1)
    Cn = D * 3 * a.n_speeds
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    frames = max(a.rollout, 1)

    def measure(first, S, steps, warmup, cost_mode=None):
        """One timed run over this rank's shard: W untimed steps, then K steps bracketed by a
        barrier + device synchronisation on both sides; returns (max-over-ranks seconds, per-kernel
        ms and launches of this rank, the resident scenes)."""
        m.reserve(local, S * D)
        p = ppamd.default_params(n_speeds=a.n_speeds, n_points=a.n_points,
                                 cost_mode=prm.cost_mode if cost_mode is None else cost_mode,
                                 emit_paths=a.emit_paths, n_draws=a.draws,
                                 noise_first_scene=first,
                                 speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if a.n_speeds == 8 else None)
        traffic = None
        if a.rollout:
            scenes, traffic = ppamd.synth_traffic(m, S, seed=a.seed, first=first, device=local, stream=sp)
        else:
            scenes = ppamd.synth_device(m, S, seed=a.seed, first=first, device=local, stream=sp)
        res = ppamd.alloc_result(S, p, xp="torch", device=dev)
        torch.cuda.synchronize(dev)

        def step():
            if a.rollout:
                ppamd.rollout(m, scenes, traffic, p, res, a.rollout, 3, a.sensor_range, device=local, stream=sp)
            else:
                ppamd.evaluate(m, scenes, p, res, device=local, stream=sp)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        # the timed region records K2's events only (each event costs a few us of stream time; the
        # roofline needs K2's launch duration), every kernel's in a short pass after it
        m.timing(local, ppamd.TIMING_K2)
        m.read_timing(local)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        ms, launches = m.read_timing(local)
        m.timing(local, ppamd.TIMING_ALL)
        for _ in range(min(steps, 5)):
            step()
        torch.cuda.synchronize(dev)
        ms_all, launches_all = m.read_timing(local)
        m.timing(local, False)
        del res
        return max_over_ranks(elapsed, dist), (ms, launches, ms_all, launches_all), scenes

    if a.scaling == "strong":
        first, S = shard(rank, world, total=a.scenes)
        total_scenes = a.scenes
    else:
        first, S = shard(rank, world, per_rank=a.scenes)
        total_scenes = a.scenes * world
    elapsed, (ms, launches, ms_all, launches_all), scenes = measure(first, S, a.steps, a.warmup)
    value = total_scenes * Cn * a.steps * frames / elapsed
    # per-rank kernel times (HIP events on each rank's launch streams): k_cand from the timed
    # region, every kernel from the short pass after it
    kms = {"rank": rank, "scenes": S, "k_prep": (ms_all[0] / launches_all[0]) if launches_all[0] else None,
           "k_cand": ms[1] / max(launches[1], 1),
           "k_out": (ms_all[2] / launches_all[2]) if launches_all[2] else None,
           "k_cand_breakdown_pass": ms_all[1] / max(launches_all[1], 1)}
    per_rank = [kms]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, kms)
    pcie = None
    if not (a.no_pcie or a.rollout or a.emit_paths or D > 1):
        # side measurement, never `value`: the same batch handed over in pinned host buffers, every
        # rank its own shard through its own link; the job's step is the slowest rank's median step
        if dist:
            dist.barrier()
        try:
            hp, _ = host_pipeline(m, scenes, prm, local, a.pcie_chunks, a.steps, min(a.warmup, 2))
            err = None
        except Exception as ex:         # a side measurement never takes the bench line down
            hp, err = None, f"{type(ex).__name__}: {ex}"
        # every rank reaches the MAX (a failed rank reports inf), so no rank waits for a lost peer
        ms_max = max_over_ranks(hp["ms_per_step"] if hp else float("inf"), dist)
        if hp is None or ms_max == float("inf"):
            pcie = {"error": err or "failed on another rank"}
        else:
            pcie = {"value": total_scenes * Cn / (ms_max * 1e-3), "unit": "candidate trajectories/s",
                    "ms_per_step": ms_max, "ms_per_step_mean": hp["ms_per_step_mean"],
                    "ms_per_step_min": hp["ms_per_step_min"], "chunks": hp["chunks"],
                    "h2d_bytes_per_step": hp["h2d_bytes_per_step"] * world,
                    "d2h_bytes_per_step": hp["d2h_bytes_per_step"] * world,
                    "pcie_gb_per_s_per_gpu": hp["pcie_gb_per_s"],
                    "h2d_only_gb_per_s": hp["h2d_only_gb_per_s"],
                    "d2h_only_gb_per_s": hp["d2h_only_gb_per_s"],
                    "what": "scenes in pinned host memory, H2D + pp_eval + D2H of winner, n_out, next_x/y, "
                            "costs, status; chunks pipelined over 3 streams; per-rank figures are rank 0's"}
    weak = None
    if world > 1 and not a.no_weak and a.scaling == "strong":
        del scenes
        torch.cuda.empty_cache()
        wfirst, wS = shard(rank, world, per_rank=CONFIG5_SCENES)
        wel, _, scenes = measure(wfirst, wS, a.steps, a.warmup)
        weak = {"value": wS * world * Cn * a.steps * frames / wel, "scenes_per_gpu": wS,
                "ms_per_step": wel / a.steps * 1e3}
    # dominant kernel: k_cand on this rank
    k_cand_ms = kms["k_cand"]
    bpc = algorithmic_bytes_per_candidate(Cn, a.n_points, a.emit_paths)
    # K2 stages per step (1: pp_eval times a split batch's overlapping parts as one stage, the span
    # from the first part's K2 start to the last part's K2 end)
    k2_per_step = max(launches[1] // max(a.steps * frames, 1), 1)
    cands_launch = S * Cn // k2_per_step
    achieved = bpc * cands_launch / (k_cand_ms * 1e-3) / 1e9
    pmc = pmc_for(load_pmc_all(), S, Cn, a.n_points, a.emit_paths, D, a.comfort)
    # the same fraction from the profiler's average K2 duration of this exact launch shape (a
    # committed rocprofv3 run of this command; durations do not carry over between batch sizes)
    rp = load_rocprof_all().get(pmc_tag(S, Cn, a.n_points, a.emit_paths, D, a.comfort))
    rp = rp if rp and rp.get("launches_per_step") == k2_per_step and not a.rollout else None
    # counters and profiler durations of another library build describe another binary: dropped
    pmc, rp, stamp = profile_entries(pmc, rp, ppamd.lib_sha256())
    traffic, traffic_pipe = roofline_fields(pmc, cands_launch, bpc, k_cand_ms)
    # the small-batch shapes run the whole step in one launch: its events time K1 + K2 + K4
    fused_step = bool(launches_all[1]) and not launches_all[0] and not a.rollout
    wname = workload_name(S, Cn, a.n_speeds, a.n_points, a.emit_paths, D, a.rollout)
    out = {
        "metric": "candidate trajectories/sec (spline+cost, 50-pt horizon) at 1/2/4/8 MI355X",
        "value": value, "unit": "candidate trajectories/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": a.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (Philox scenes on highway_map.csv, seeded; SURVEY.md §8(d))",
        "config": {"workload": (f"{wname}: {total_scenes} scenes x {D} sensor-noise draws x 3 lanes x "
                                f"{a.n_speeds} speeds, per-scene argmin over draws" if D > 1 else
                                f"{wname}: {total_scenes} scenes x 3 lanes x {a.n_speeds} speeds")
                               + workload_scope(wname, S, total_scenes, world, a.scaling)
                               + f", {a.n_points}-pt horizon"
                               + (", all paths emitted" if a.emit_paths else ", winner path + costs")
                               + (f", closed loop: {a.rollout} frames per step (plan + simulator, 3 points "
                                  f"driven per frame, sensor range {a.sensor_range:g} m)" if a.rollout else "")
                               + (", comfort cost" if a.comfort else ", reference decision"),
                   "scenes_total": total_scenes, "scenes_per_gpu": S, "candidates_per_scene": Cn,
                   "horizon_points": a.n_points,
                   "parallelism": f"contiguous scene shards x{world}, no collective (gloo barrier + max for timing)",
                   **({"debug": dict(kv.partition("=")[::2] for kv in a.debug), "reportable": False}
                      if a.debug else {})},
        "kernels_ms_avg": {k: kms[k] for k in ("k_prep", "k_cand", "k_out")},
        "kernels_ms_source": ("k_cand: HIP events around each K2 launch in the timed region (the only events "
                              "there); k_prep, k_out: every kernel's events in a pass of min(steps, 5) steps "
                              "after it"),
        "per_rank_kernels_ms": per_rank,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel_ms": k_cand_ms, "launches_per_step": k2_per_step,
                     "kernel_time_source": ("the whole one-launch step (K1 + K2 + K4 in one kernel: its "
                                            "dispatch's own start/end events), timed region" if fused_step else
                                            "HIP events around each K2 launch on its own stream, timed region "
                                            "(a batch split over streams: the span of its parts' K2 launches)"),
                     "profile_stamp": stamp,
                     "frac_rocprof": (bpc * cands_launch / (rp["dominant_ms_per_launch"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                                      if rp else None),
                     "kernel_ms_rocprof": rp["dominant_ms_per_launch"] if rp else None,
                     "rocprof_source": rp["source"] if rp else None,
                     "kernel": ", ".join(pmc["kernels"]) if pmc and pmc.get("kernels") else "k_cand",
                     "algorithmic_bytes_per_candidate": bpc,
                     "traffic_pipeline": traffic_pipe,
                     "traffic_source": (pmc or {}).get("source"),
                     "traffic_profiled_launch": ({k: pmc.get(k) for k in ("scenes", "candidates_per_scene", "n_points",
                                                                           "candidates_per_launch", "kernels")}
                                                 if pmc else None)},
    }
    if weak:
        out["weak_scaling"] = weak
    if pcie:
        out["pcie_inclusive"] = pcie
    # the bound that matters for this path: FP64 VALU issue (no MFMA-shaped work, HBM a few %)
    peak, peak_add = load_valu_peak()
    if pmc and peak:
        c = pmc["counters"]
        pc = pmc["candidates_per_launch"]
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")) / pc * cands_launch
        allv = c.get("SQ_INSTS_VALU", 0.0) / pc * cands_launch
        ach = f64 / (k_cand_ms * 1e-3)
        out["valu_roofline"] = {"bound": "fp64-valu-issue", "kernel": "k_cand",
                                "achieved_f64_wave_instr_per_s": ach, "peak_f64_fma_wave_instr_per_s": peak,
                                "frac": ach / peak, "all_valu_wave_instr_per_launch": allv,
                                "f64_wave_instr_per_launch": f64,
                                "all_valu_wave_instr_per_s": allv / (k_cand_ms * 1e-3),
                                "peak_issue_wave_instr_per_s": peak_add,
                                "issue_frac": allv / (k_cand_ms * 1e-3) / peak_add if peak_add else None,
                                "source": "rocprofv3 PMC SQ_INSTS_VALU_* per candidate (profiles/pmc_summary.json) "
                                          "x this launch's candidates / this run's k_cand time; peak measured by "
                                          "tools/valu_peak.hip"}
    if a.rollout:
        out["scene_frames_per_s"] = total_scenes * a.steps * frames / elapsed
    if (world == 1 and a.scaling == "strong" and wname == "BASELINE config 5" and S == CONFIG5_SCENES
            and not a.debug and not a.no_shard_projection):
        # the 2-, 4- and 8-GPU shards of the same batch, timed in this process on this GPU right
        # after the headline (same box, same build): the projected N-GPU speed-ups
        t_sh = {}
        for n in (2, 4, 8):
            el_n, _, _ = measure(0, CONFIG5_SCENES // n, a.steps, a.warmup)
            t_sh[n] = el_n / a.steps
        out["shard_projection"] = dict(shard_projection(elapsed / a.steps, t_sh), what=(
            "PROJECTION from one GPU, not a multi-GPU measurement: config 5 on N GPUs = N independent "
            "shards of 2,097,152 / N scenes (no collective); speed-up = min(t(full batch), N t(shard)) / "
            "t(shard), i.e. against the batch's best one-GPU policy (one call, or the N shards in "
            "sequence); all timed in this run (same protocol, steps and warmup)"))
    if (world == 1 and a.scaling == "strong" and wname == "BASELINE config 5" and S == CONFIG5_SCENES
            and not a.debug and not a.comfort and not a.no_comfort):
        # the data-dependent decision (north_star's "argmin per scene") on the same batch: the
        # comfort cost mode, where k_cand takes each scene's first-minimum cost and stores the
        # winner's spline, and k_winner_st re-runs the winner with outputs
        del scenes
        torch.cuda.empty_cache()
        cel, (cms, clh, cms_all, cla), scenes = measure(first, S, a.steps, a.warmup, ppamd.COST_COMFORT)
        ck = {"k_prep": cms_all[0] / cla[0] if cla[0] else None, "k_cand": cms[1] / max(clh[1], 1),
              "k_winner": cms_all[2] / cla[2] if cla[2] else None}
        cstep = cel / a.steps * 1e3
        cach = bpc * cands_launch / (ck["k_cand"] * 1e-3) / 1e9
        cpmc = pmc_for(load_pmc_all(), S, Cn, a.n_points, a.emit_paths, D, True)
        crp = load_rocprof_all().get(pmc_tag(S, Cn, a.n_points, a.emit_paths, D, True))
        crp = crp if crp and crp.get("launches_per_step") == 1 else None
        cpmc, crp, cstamp = profile_entries(cpmc, crp, ppamd.lib_sha256())
        ctraffic, cpipe = roofline_fields(cpmc, cands_launch, bpc, ck["k_cand"])
        out["comfort"] = {
            "value": total_scenes * Cn * a.steps / cel, "unit": "candidate trajectories/s",
            "ms_per_step": cstep, "kernels_ms_avg": ck,
            "k_winner_share_of_step": (ck["k_winner"] / cstep) if ck["k_winner"] else None,
            "roofline": {"bound": "hbm", "achieved": cach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": cach / HBM_PEAK_GBS, "kernel": "k_cand", "kernel_ms": ck["k_cand"],
                         "algorithmic_bytes_per_candidate": bpc, "traffic": ctraffic, "traffic_pipeline": cpipe,
                         "profile_stamp": cstamp,
                         "frac_rocprof": (bpc * cands_launch / (crp["dominant_ms_per_launch"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                                          if crp else None),
                         "kernel_ms_rocprof": crp["dominant_ms_per_launch"] if crp else None},
            "what": ("BASELINE config 5's batch under the comfort cost (cost_mode 1): per scene the first "
                     "minimum of the 15 candidate costs (k_cand, in LDS), the winner's spline slot stored, "
                     "k_winner_st re-runs it with next_x/next_y; same timing protocol as the headline; "
                     "k_prep and k_winner from the pass after the timed region")}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.rollout:
        model, nproc, share = host_cpu()
        threads = a.cpu_threads or share

        def scenes_host(start, n):
            return {k: np.ascontiguousarray(v[..., start:start + n].cpu().numpy()) for k, v in scenes.items()}
        out["cpu_baseline"] = cpu_baseline(scenes_host, S, prm, a.cpu_seconds, threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

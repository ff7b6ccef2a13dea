"""bench.py — candidate trajectories/s of the MI355X evaluator (BASELINE.json metric).

A step = one pp_eval over one resident batch of synthetic scenes (inputs already in HBM): K1 scene
prep + K2 candidate evaluation (3 lanes x n_speeds, 50-point horizon, spline + limiter + cost)
+ per-scene winner path. Default workload = BASELINE config 5's batch, 2,097,152 scenes x 15
candidates per GPU (weak scaling: rank r evaluates global scenes [r*S, (r+1)*S) of one seeded
synthetic stream; no collective on the data path, only the timing barrier + max).

Run: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "carnd-path-planning-project_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
SCENE_BYTES = 4 * 8 + 20 * 8 + 3 * 4 + 12 * (4 + 4 * 8)   # SoA scene record (include/pp.h): 636 B


def algorithmic_bytes_per_candidate(C_, N, emit_paths):
    """scene record read once per scene, winner path + n_out/winner written once
    per scene, one f64 cost per candidate; all-paths mode writes every candidate's N points."""
    if emit_paths:
        return (SCENE_BYTES + 8) / C_ + 8 + 16 * N + 4
    return (SCENE_BYTES + 8 + 16 * N) / C_ + 8


def shard(rank, scenes_per_rank):
    """Weak scaling: rank r owns global scenes [r*S, (r+1)*S) of one seeded synthetic stream
    (pp_synth_scenes first_scene = r*S); scenes depend only on (seed, global index)."""
    return rank * scenes_per_rank, scenes_per_rank


def max_over_ranks(elapsed, dist, device):
    """The job's time is the slowest rank's (MAX all-reduce; RCCL on GPUs, gloo in the CPU test)."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_valu_peak():
    """Measured FP64 VALU issue rate (tools/valu_peak.hip on the MI355X, profiles/r01_valu_peak.json)."""
    p = os.path.join(REPO, "profiles", "r01_valu_peak.json")
    try:
        j = json.load(open(p))
        return j["v_fma_f64"]["wave_instr_per_s"], j["v_add_f64"]["wave_instr_per_s"]
    except Exception:
        return None, None


def load_f64_instr(tag):
    """FP64 VALU wave-instructions per k_cand launch from the committed PMC summary."""
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        c = json.load(open(p))[tag]["counters"]
        return sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                            "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")), c.get("SQ_INSTS_VALU")
    except Exception:
        return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scenes", type=int, default=2_097_152, help="scenes per GPU")
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
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(m, scenes_dev, prm, budget_s):
    """Reference planning code (oracle/_ref, compiled from the reference's sources) if it was
    built, else the C restatement (oracle/liboracle.so), on one host core over a bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    import ppamd
    wx, wy = ppamd.highway_map()
    rlib = oracle_lib.load_ref() if prm.n_points == 50 and not prm.emit_paths and prm.n_draws <= 1 else None
    olib = None if rlib else oracle_lib.load_oracle()
    chunk = 2048
    S = int(scenes_dev["ego_x"].shape[0])
    done, t_used, start = 0, 0.0, 0
    offs = [prm.speed_offsets[i] for i in range(prm.n_speeds - 1)]
    while t_used < budget_s and start < S:
        host = {k: np.ascontiguousarray(v[..., start:start + chunk].cpu().numpy()) for k, v in scenes_dev.items()}
        t0 = time.perf_counter()
        if rlib:
            oracle_lib.ref_eval(rlib, wx, wy, host, prm.n_speeds, offs, with_frame=False)
        else:
            oracle_lib.oracle_eval(olib, wx, wy, host, prm, info=False)
        t_used += time.perf_counter() - t0
        done += host["ego_x"].shape[0]
        start += chunk
    cands = done * 3 * prm.n_speeds * max(prm.n_draws, 1)
    return {"value": cands / t_used, "unit": "candidate trajectories/s", "cores": 1,
            "kind": "reference" if rlib else "port",
            "sample": f"first {done} scenes x {3 * prm.n_speeds * max(prm.n_draws, 1)} candidates of the same synthetic "
                      f"batch ({t_used:.1f} s, single thread; "
                      + ("reference src/main.cpp classes built by oracle/Makefile" if rlib else
                         "C restatement oracle/pp_oracle.c") + ")"}


def load_traffic(tag):
    """Per-launch HBM bytes of k_cand from the committed rocprofv3 PMC summary (profiles/)."""
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        e = d.get(tag)
        if not e:
            return None, None
        return e["hbm_bytes_per_launch"], e.get("source")
    except Exception:
        return None, None


def main():
    a = parse()
    import torch
    import ppamd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    S = a.scenes
    prm = ppamd.default_params(n_speeds=a.n_speeds, n_points=a.n_points,
                               cost_mode=ppamd.COST_COMFORT if a.comfort else ppamd.COST_REFERENCE,
                               emit_paths=a.emit_paths, n_draws=a.draws, noise_first_scene=0,
                               speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if a.n_speeds == 8 else None)
    D = max(a.draws, 1)
    Cn = D * 3 * a.n_speeds
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    m.reserve(local, S * D)
    first, _ = shard(rank, S)
    prm.noise_first_scene = first
    traffic = None
    if a.rollout:
        scenes, traffic = ppamd.synth_traffic(m, S, seed=a.seed, first=first, device=local, stream=sp)
    else:
        scenes = ppamd.synth_device(m, S, seed=a.seed, first=first, device=local, stream=sp)
    res = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    torch.cuda.synchronize(dev)

    def step():
        if a.rollout:
            ppamd.rollout(m, scenes, traffic, prm, res, a.rollout, 3, a.sensor_range, device=local, stream=sp)
        else:
            ppamd.evaluate(m, scenes, prm, res, device=local, stream=sp)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    m.timing(local, True)
    m.read_timing(local)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms, launches = m.read_timing(local)
    m.timing(local, False)
    elapsed = max_over_ranks(elapsed, dist, dev)
    frames = max(a.rollout, 1)
    total_cands = S * Cn * world * a.steps * frames
    value = total_cands / elapsed
    # dominant kernel: k_cand (HIP events on the launch stream, timed region only)
    k_cand_ms = ms[1] / max(launches[1], 1)      # per launch (one frame)
    bpc = algorithmic_bytes_per_candidate(Cn, a.n_points, a.emit_paths)
    bytes_launch = bpc * S * Cn
    achieved = bytes_launch / (k_cand_ms * 1e-3) / 1e9
    tag = f"k_cand_S{S}_C{Cn}_N{a.n_points}" + ("_paths" if a.emit_paths else "") + (f"_D{D}" if D > 1 else "")
    traffic, traffic_src = load_traffic(tag)
    out = {
        "metric": "candidate trajectories/sec (spline+cost, 50-pt horizon) at 1/2/4/8 MI355X",
        "value": value, "unit": "candidate trajectories/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (Philox scenes on highway_map.csv, seeded; SURVEY.md §8(d))",
        "config": {"workload": (f"BASELINE config 4: {S} scenes x {D} sensor-noise draws x 3 lanes x "
                                f"{a.n_speeds} speeds, per-scene argmin over draws" if D > 1 else
                                f"BASELINE config 5 batch: {S} scenes x 3 lanes x {a.n_speeds} speeds")
                               + f", {a.n_points}-pt horizon per GPU"
                               + (", all paths emitted" if a.emit_paths else ", winner path + costs")
                               + (f", closed loop: {a.rollout} frames per step (plan + simulator, 3 points "
                                  f"driven per frame, sensor range {a.sensor_range:g} m)" if a.rollout else "")
                               + (", comfort cost" if a.comfort else ", reference decision"),
                   "scenes_per_gpu": S, "candidates_per_scene": Cn, "horizon_points": a.n_points,
                   "parallelism": f"scene shards x{world}, no collective"},
        "kernels_ms_avg": {"k_prep": ms[0] / max(launches[0], 1), "k_cand": k_cand_ms,
                           "k_out": (ms[2] / launches[2]) if launches[2] else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "k_cand", "algorithmic_bytes_per_candidate": bpc,
                     "traffic_source": traffic_src},
    }
    # the bound that matters for this path: FP64 VALU issue (no MFMA-shaped work, HBM ~3 %)
    f64, allv = load_f64_instr(tag)
    peak, peak_add = load_valu_peak()
    if f64 and peak:
        ach = f64 / (k_cand_ms * 1e-3)
        out["valu_roofline"] = {"bound": "fp64-valu-issue", "kernel": "k_cand",
                                "achieved_f64_wave_instr_per_s": ach, "peak_f64_fma_wave_instr_per_s": peak,
                                "frac": ach / peak, "all_valu_wave_instr_per_launch": allv,
                                "f64_wave_instr_per_launch": f64,
                                "source": "rocprofv3 PMC SQ_INSTS_VALU_*_F64 per launch (profiles/pmc_summary.json) "
                                          "/ this run's k_cand time; peak measured by tools/valu_peak.hip"}
        if allv and peak_add:
            # every VALU instruction (FP64, int, moves, compares) against the fastest measured
            # single-instruction issue rate (v_add_f64): the share of the VALU issue slots used
            out["valu_roofline"]["all_valu_wave_instr_per_s"] = allv / (k_cand_ms * 1e-3)
            out["valu_roofline"]["peak_issue_wave_instr_per_s"] = peak_add
            out["valu_roofline"]["issue_frac"] = allv / (k_cand_ms * 1e-3) / peak_add
    if a.rollout:
        out["scene_frames_per_s"] = S * world * a.steps * frames / elapsed
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not a.rollout:
        out["cpu_baseline"] = cpu_baseline(m, scenes, prm, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

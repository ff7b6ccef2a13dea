"""Workgroup timeline of k_prep and k_cand<false> (diagnostic builds, -DPP_TRACE).

Build: tools/variants.sh trace "-DPP_TRACE"; run on the GPU box:
  PPAMD_LIB=$PWD/carnd-path-planning-project_amd/ppamd/libppamd_var_trace.so \
      python tools/trace_blocks.py --scenes 262144 --out gpurun_out/trace_262144
Each traced workgroup records (100 MHz constant clock) its start, the end of k_cand's phase A,
each wave's end of phase B (k_prep: each wave's end), its end and its CU. The summary splits a
kernel's span into the dispatch ramp, the steady part and the tail, and gives the block-slot and
wave-slot occupancy (how much of resident capacity x span held a block / a running wave).
Raw words go to <out>.npz for offline analysis; the summary is printed as JSON.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "carnd-path-planning-project_amd"))
K1_BASE = 3 << 16
MAXB = 1 << 18
TICK_US = 0.01          # 100 MHz


def summarize(t, waves, slots_per_cu, name):
    """t: [B, 8] words of one kernel (B blocks)."""
    t0 = t[:, 0].astype(np.int64)
    wend = t[:, 2:2 + waves].astype(np.int64)
    tend = t[:, 6].astype(np.int64) if name == "k_cand" else wend.max(1)
    T0 = t0.min()
    span = (tend.max() - T0) * TICK_US
    hw = t[:, 7]
    cu = (hw >> 32) * 4096 + (hw & 0xFFFF)        # XCC id, HW_ID low bits (wave/simd/cu/sh/se)
    cu_key = (hw >> 32) * 65536 + ((hw >> 8) & 0xF) * 256 + ((hw >> 12) & 0x1) * 16 + ((hw >> 13) & 0x7)
    ncu = len(np.unique(cu_key))
    dur = (tend - t0) * TICK_US
    start = (t0 - T0) * TICK_US
    busy_blocks = dur.sum()
    slots = ncu * slots_per_cu
    out = {"kernel": name, "blocks": int(len(t)), "cus_seen": int(ncu), "span_us": float(span),
           "block_us_mean": float(dur.mean()), "block_us_p10_p50_p90": [float(x) for x in np.percentile(dur, [10, 50, 90])],
           "block_slot_occupancy": float(busy_blocks / (slots * span)),
           "first_round_start_us_p50_p100": [float(np.percentile(np.sort(start)[:slots], 50)),
                                             float(np.sort(start)[min(slots, len(start)) - 1])],
           "last_block_start_us": float(start.max()),
           "tail_us": float(span - np.percentile((tend - T0) * TICK_US, 50 if len(t) <= slots else 99))}
    wdur = (wend - t0[:, None]) * TICK_US
    out["wave_slot_occupancy_in_blocks"] = float(wdur.sum() / (dur.sum() * waves))
    if name == "k_cand":
        pa = (t[:, 1].astype(np.int64) - t0) * TICK_US
        out["phase_a_us_mean"] = float(pa.mean())
        out["phase_a_share_of_block"] = float(pa.sum() / dur.sum())
        out["wave0_phase_b_us_mean"] = float(((wend[:, 0] - t[:, 1].astype(np.int64)) * TICK_US).mean())
        out["other_waves_phase_b_us_mean"] = float(((wend[:, 1:] - t[:, 1:2].astype(np.int64)) * TICK_US).mean())
        out["block_wait_on_last_wave_us_mean"] = float(((wend.max(1) - wend.mean(1)) * TICK_US).mean())
    # rounds: blocks started in time order; capacity `slots`
    order = np.argsort(t0)
    if len(t) > slots:
        rounds = len(t) / slots
        out["rounds"] = float(rounds)
        out["us_per_round"] = float(span / rounds)
    out["timeline_occupancy_10bins"] = occupancy_bins(t0 - T0, tend - T0, span / TICK_US, slots)
    return out


def occupancy_bins(a, b, span_ticks, slots, nb=10):
    edges = np.linspace(0, span_ticks, nb + 1)
    occ = []
    for i in range(nb):
        lo, hi = edges[i], edges[i + 1]
        ov = np.clip(np.minimum(b, hi) - np.maximum(a, lo), 0, None).sum()
        occ.append(round(float(ov / (slots * (hi - lo))), 3))
    return occ


def main():
    import torch
    import ppamd
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=262144)
    ap.add_argument("--n-speeds", type=int, default=5)
    ap.add_argument("--n-points", type=int, default=50)
    ap.add_argument("--emit-paths", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    S = a.scenes
    lib = C.CDLL(ppamd.LIB_PATH)
    lib.pp_trace_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int64]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params(n_speeds=a.n_speeds, n_points=a.n_points, emit_paths=a.emit_paths,
                               speed_offsets=[-6, -4, -3, -2, -1, 0, 2] if a.n_speeds == 8 else None)
    scenes = ppamd.synth_device(m, S, seed=0x5EED0001, device=0)
    res = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
    buf = np.zeros(8 * MAXB, np.uint64)
    summaries = []
    for rep in range(a.reps):
        ppamd.evaluate(m, scenes, prm, res, device=0)
        torch.cuda.synchronize()
        assert lib.pp_trace_read(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), buf.size) == 0
        t = buf.reshape(MAXB, 8)
        C_ = 3 * a.n_speeds
        spb = {15: 17, 24: 8}.get(C_, max(1, 256 // C_))
        nb = (S + spb - 1) // spb
        threads = ((spb * C_ + 63) // 64) * 64
        kc = t[:min(nb, K1_BASE)].copy()
        kp = t[K1_BASE:K1_BASE + (S + 255) // 256].copy()
        sp = summarize(kp, 4, 4, "k_prep")
        sc = summarize(kc, threads // 64, 4, "k_cand")
        sc["gap_prep_end_to_cand_start_us"] = float((kc[:, 0].astype(np.int64).min() -
                                                     kp[:, 2:6].astype(np.int64).max()) * TICK_US)
        summaries.append({"rep": rep, "k_prep": sp, "k_cand": sc})
        if a.out and rep == a.reps - 1:
            np.savez_compressed(a.out + ".npz", k_cand=kc, k_prep=kp)
    print(json.dumps({"scenes": S, "n_speeds": a.n_speeds, "n_points": a.n_points,
                      "emit_paths": a.emit_paths, "runs": summaries}, indent=1))


if __name__ == "__main__":
    main()

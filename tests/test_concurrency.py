"""Concurrent callers of one map (INTEGRATION.md "Batched use": each stream that calls pp_eval gets
its own workspace, and the map's lock is held from binding the workspace through the asynchronous
launches; pp_plan_batch_host stages through its own pinned buffers under a per-device lock).

Host threads evaluate different batches on their own streams at the same time: reference,
comfort and all-paths modes, batch sizes from 1 scene to 524,288 (the one-stream path, the
multi-stream split, the fused small-batch step), each thread's sizes in an order that grows and
shrinks its stream's workspace between calls, three rounds each; one more thread runs
pp_plan_batch_host on host scenes meanwhile. Every result equals the same batch evaluated alone
beforehand, bit for bit (the library's own outputs are NaN-poisoned at every call under the GPU
suite's PP_DBG_POISON, tests/conftest.py, so a result cannot be left over from the serial run)."""
import threading

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

pytestmark = pytest.mark.gpu
OFFS8 = [-6, -4, -3, -2, -1, 0, 2]
PLAN = [[(3001, "ref"), (262_144, "ref"), (70_001, "comfort")],
        [(150_001, "comfort"), (4096, "ref"), (9000, "paths")],
        [(20_000, "paths"), (131_073, "ref"), (1, "ref")],
        [(524_288, "ref"), (257, "comfort"), (65_537, "ref")]]
ROUNDS = 3


def same(torch, a, b):
    if a.is_floating_point():
        return torch.equal(torch.nan_to_num(a, nan=7e7), torch.nan_to_num(b, nan=7e7))
    return torch.equal(a, b)


def test_concurrent_streams_equal_serial():
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    dev = torch.device("cuda", 0)
    prms = {"ref": ppamd.default_params(), "comfort": ppamd.default_params(cost_mode=ppamd.COST_COMFORT),
            "paths": ppamd.default_params(n_speeds=8, n_points=100, speed_offsets=OFFS8, emit_paths=True)}
    jobs = []                      # per thread: (S, params key, scenes, serial result, result buffer)
    for t, lst in enumerate(PLAN):
        jt = []
        for j, (S, pk) in enumerate(lst):
            sc = ppamd.synth_device(m, S, seed=0xC0C0 + 16 * t + j, device=0)
            ref = ppamd.alloc_result(S, prms[pk], xp="torch", device=dev)
            ppamd.evaluate(m, sc, prms[pk], ref, device=0)
            jt.append((S, pk, sc, ref, ppamd.alloc_result(S, prms[pk], xp="torch", device=dev)))
        jobs.append(jt)
    host = ppamd.synth_host(m, 5000, seed=0xC0C1)
    host_ref = ppamd.plan_batch_host(m, host, prms["ref"])
    torch.cuda.synchronize()

    errors, checked = [], [0] * (len(PLAN) + 1)

    def device_worker(t):
        try:
            st = torch.cuda.Stream(dev)
            for rnd in range(ROUNDS):
                order = jobs[t] if rnd % 2 == 0 else jobs[t][::-1]
                for S, pk, sc, ref, got in order:
                    ppamd.evaluate(m, sc, prms[pk], got, device=0, stream=st.cuda_stream)
                    st.synchronize()
                    for k in ref:
                        if not same(torch, got[k], ref[k]):
                            errors.append(f"thread {t} round {rnd}: {S} scenes ({pk}) field {k} differs")
                    checked[t] += 1
        except Exception as ex:                    # reported by the main thread
            errors.append(f"thread {t}: {type(ex).__name__}: {ex}")

    def host_worker():
        try:
            for rnd in range(ROUNDS):
                r = ppamd.plan_batch_host(m, host, prms["ref"])
                for k, v in host_ref.items():
                    a, b = np.ascontiguousarray(r[k]), np.ascontiguousarray(v)
                    if a.tobytes() != b.tobytes():
                        errors.append(f"plan_batch_host round {rnd}: field {k} differs")
                checked[-1] += 1
        except Exception as ex:
            errors.append(f"plan_batch_host: {type(ex).__name__}: {ex}")

    threads = [threading.Thread(target=device_worker, args=(t,)) for t in range(len(PLAN))]
    threads.append(threading.Thread(target=host_worker))
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=150)
    assert not any(th.is_alive() for th in threads), "a caller thread did not finish"
    assert not errors, errors[:10]
    assert checked == [ROUNDS * len(l) for l in PLAN] + [ROUNDS]
    print(f"{len(PLAN)} device threads x {ROUNDS} rounds x 3 batches + pp_plan_batch_host x {ROUNDS}: "
          f"every result bit-identical to the serial evaluation")

"""Multi-process path on CPU (gloo, world_size 2): the bench's scene sharding and max-over-ranks
timing. Each rank synthesises its shard, evaluates it with the CPU oracle, and rank 0 checks that
the gathered shards equal a single-process evaluation of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib
from oracle_lib import ppamd

S_PER_RANK = 48


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    first, n = bench.shard(rank, world, per_rank=S_PER_RANK)
    sc = ppamd.synth_host(m, n, seed=99, first=first)
    prm = ppamd.default_params()
    r = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, sc, prm, info=False)
    cost = torch.from_numpy(r["cost"]).contiguous()
    nxt = torch.from_numpy(np.ascontiguousarray(r["next_x"].T))
    gc = [torch.zeros_like(cost) for _ in range(world)]
    gn = [torch.zeros_like(nxt) for _ in range(world)]
    dist.all_gather(gc, cost)
    dist.all_gather(gn, nxt)
    t = bench.max_over_ranks(1.0 + rank, dist)
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"), cost=torch.cat(gc).numpy(),
                 next_x=torch.cat(gn).numpy(), t=t)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_process(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    z = np.load(tmp_path / "dist.npz")
    assert float(z["t"]) == 2.0                       # max over ranks
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    full = ppamd.synth_host(m, world * S_PER_RANK, seed=99, first=0)
    r = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, full, ppamd.default_params(), info=False)
    assert np.array_equal(z["cost"], r["cost"])
    assert np.array_equal(z["next_x"], r["next_x"].T)


def test_shard_arithmetic():
    """Strong scaling (BASELINE config 5: 2,097,152 scenes in total) and weak scaling shards for
    1/2/4/8 GPUs: contiguous, disjoint, covering, balanced."""
    import bench
    for G in (1, 2, 4, 8):
        sh = [bench.shard(r, G, total=bench.CONFIG5_SCENES) for r in range(G)]
        assert sh[0][0] == 0 and sum(n for _, n in sh) == bench.CONFIG5_SCENES
        assert all(sh[i][0] + sh[i][1] == sh[i + 1][0] for i in range(G - 1))
        assert {n for _, n in sh} == {bench.CONFIG5_SCENES // G}
        w = [bench.shard(r, G, per_rank=1000) for r in range(G)]
        assert w == [(1000 * r, 1000) for r in range(G)]
    odd = [bench.shard(r, 3, total=10) for r in range(3)]
    assert odd == [(0, 3), (3, 3), (6, 4)]
    envs = bench.rank_envs(4, 12345, base={})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"] and all(e["WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


def test_launcher_starts_n_ranks():
    """`bench.py --gpus 4` without torchrun starts 4 rank processes (gloo barrier + max); the CPU
    rehearsal evaluates each rank's shard with the oracle and reports n_gpus = 4 over the whole
    batch, equal to a single-process evaluation."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(oracle_lib.REPO, "bench.py"), "--gpus", "4", "--cpu-ranks",
                        "--scenes", "66", "--steps", "1"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 4 and out["scaling"] == "strong"
    assert [tuple(x) for x in out["shards"]] == [(0, 16), (16, 17), (33, 16), (49, 17)]
    wx, wy = ppamd.highway_map()
    m = ppamd.Map(wx, wy)
    full = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, ppamd.synth_host(m, 66, seed=0x5EED0001, first=0),
                                  ppamd.default_params(), info=False)
    parts = [float(np.nansum(full["cost"][f:f + n])) for f, n in out["shards"]]
    assert np.allclose(parts, out["cost_digests"], rtol=1e-12)


@pytest.mark.gpu
def test_launcher_two_ranks_on_the_gpu():
    """`bench.py --gpus 2` on the GPU box: two rank processes (more ranks than GPUs share them), the
    strong-scaling shards of one batch, gloo barrier + MAX, the PCIe leg on every rank, and the
    weak-scaling side measurement; rank 0 reports n_gpus = 2 and both ranks' kernel times."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(oracle_lib.REPO, "bench.py"), "--gpus", "2", "--scenes", "65536",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--pcie-chunks", "2"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["value"] > 0
    ranks = out["per_rank_kernels_ms"]
    assert [x["rank"] for x in ranks] == [0, 1] and [x["scenes"] for x in ranks] == [32768, 32768]
    assert all(x["k_cand"] > 0 for x in ranks)
    assert out["weak_scaling"]["scenes_per_gpu"] == bench_config5() and out["weak_scaling"]["value"] > 0
    assert out["pcie_inclusive"]["value"] > 0, out["pcie_inclusive"]


def bench_config5():
    import bench
    return bench.CONFIG5_SCENES

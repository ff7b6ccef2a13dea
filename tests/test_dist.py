"""Multi-process path on CPU (gloo, world_size 2): the bench's scene sharding and max-over-ranks
timing. Each rank synthesises its shard, evaluates it with the CPU oracle, and rank 0 checks that
the gathered shards equal a single-process evaluation of the whole batch."""
import os
import socket

import numpy as np
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
    first, n = bench.shard(rank, S_PER_RANK)
    sc = ppamd.synth_host(m, n, seed=99, first=first)
    prm = ppamd.default_params()
    r = oracle_lib.oracle_eval(oracle_lib.load_oracle(), wx, wy, sc, prm, info=False)
    cost = torch.from_numpy(r["cost"]).contiguous()
    nxt = torch.from_numpy(np.ascontiguousarray(r["next_x"].T))
    gc = [torch.zeros_like(cost) for _ in range(world)]
    gn = [torch.zeros_like(nxt) for _ in range(world)]
    dist.all_gather(gc, cost)
    dist.all_gather(gn, nxt)
    t = bench.max_over_ranks(1.0 + rank, dist, torch.device("cpu"))
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

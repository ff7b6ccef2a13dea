"""bench.py's PCIe-inclusive side measurement: the batch handed over in pinned host
buffers, cut into chunks whose H2D copy, pp_eval and D2H copy overlap on three streams. The chunk
arithmetic is checked on the CPU; on the GPU the host-side outputs must equal the resident
(HBM-in, HBM-out) evaluation of the same batch bit for bit, ragged last chunk included."""
import numpy as np
import pytest

import bench
import oracle_lib
from oracle_lib import ppamd


@pytest.mark.parametrize("S,k", [(10, 3), (4096, 4), (7, 7), (5, 8), (1, 4), (2_097_152, 4)])
def test_chunk_bounds_cover_batch(S, k):
    b = bench.chunk_bounds(S, k)
    assert b[0][0] == 0 and b[-1][1] == S
    assert all(lo < hi for lo, hi in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    sizes = [hi - lo for lo, hi in b]
    assert max(sizes) - min(sizes) <= 1
    assert len(b) == min(k, S)


@pytest.mark.gpu
@pytest.mark.parametrize("S,chunks", [(1000, 3), (4099, 4)])
def test_host_pipeline_equals_resident(S, chunks):
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    prm = ppamd.default_params()
    scenes = ppamd.synth_device(m, S, seed=77, first=123_456, device=0)
    res = ppamd.alloc_result(S, prm, xp="torch", device=torch.device("cuda", 0))
    ppamd.evaluate(m, scenes, prm, res, device=0)
    torch.cuda.synchronize()
    ref = ppamd.result_to_numpy(res)
    stats, outs = bench.host_pipeline(m, scenes, prm, 0, chunks, steps=2, warmup=1)
    assert stats["chunks"] == chunks
    for f in bench.OUT_FIELDS:
        got = outs[f].numpy()
        want = ref[f]
        if f == "status":
            got = got.view(np.uint32)
        assert got.shape == want.shape, f
        assert np.array_equal(np.ascontiguousarray(got).view(np.uint8),
                              np.ascontiguousarray(want).view(np.uint8)), f

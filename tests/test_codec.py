"""Wire codec: pp_telemetry_parse / pp_control_format against the
reference's own hasData + nlohmann::json (oracle/_ref/libppref_json.so) — through the committed
fixture tests/golden/codec_golden.npz everywhere, and live on fresh corpora where the reference
build exists. Every value is compared bit for bit, every control message byte for byte."""
import numpy as np
import pytest

import codec_corpus
import oracle_lib
from oracle_lib import ppamd

G = np.load(oracle_lib.GOLDEN + "/codec_golden.npz")


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def same_status(ours, ref):
    # ours: 0 ok / 2 ok but more cars than columns -> ref 0; 1 -> 1; -1 -> -1
    return (ref == 0 and ours in (0, 2)) or ours == ref


def check_frame(d, st, s, ref):
    rs, ego, px, py, npv, ids, cars = ref
    assert same_status(int(st[s]), rs), (s, int(st[s]), rs)
    if rs != 0:
        return
    got_ego = np.array([d["ego_x"][s], d["ego_y"][s], d["ego_yaw_deg"][s], d["ego_speed_mph"][s]])
    assert (bits(got_ego) == bits(ego)).all(), s
    assert int(d["n_prev"][s]) == npv
    k = min(npv, 10)
    assert (bits(d["prev_x"][:k, s]) == bits(px[:k])).all() and (bits(d["prev_y"][:k, s]) == bits(py[:k])).all(), s
    nc = int(d["n_cars"][s])
    assert nc == min(len(ids), d["car_id"].shape[0]), s
    assert (d["car_id"][:nc, s] == ids[:nc]).all(), s
    got = np.stack([d["car_x"][:nc, s], d["car_y"][:nc, s], d["car_vx"][:nc, s], d["car_vy"][:nc, s]], -1)
    assert (bits(got) == bits(cars[:nc])).all(), s


def golden_msgs():
    buf = G["msg_buf"].tobytes()
    off = G["msg_off"]
    return [buf[off[i]:off[i + 1]] for i in range(len(off) - 1)]


@pytest.mark.parametrize("threads", [1, 8])
def test_parse_matches_reference_fixture(threads):
    msgs = golden_msgs()
    d, st = ppamd.telemetry_parse(msgs, threads=threads)
    for s in range(len(msgs)):
        n = int(G["n_cars"][s])
        ref = (int(G["status"][s]), G["ego"][s], G["prev_x"][s], G["prev_y"][s], int(G["n_prev"][s]),
               G["car_id"][s][:n], G["cars"][s][:n])
        check_frame(d, st, s, ref)
    assert (st == 0).sum() > 300 and (st == 1).sum() > 5 and (st == 3).sum() > 5 and (st == -1).sum() > 5


def test_format_matches_reference_fixture():
    vals = G["values"]
    buf, off = G["dump_buf"].tobytes(), G["dump_off"]
    starts = list(range(0, len(vals) - 50, 7))
    xs = np.stack([vals[k:k + 50] for k in starts], 1)           # point-major [N][S]
    ys = np.stack([vals[::-1][k:k + 50] for k in starts], 1)
    got = ppamd.control_format(xs, ys, np.full(len(starts), 50, np.int32))
    for i in range(len(starts)):
        assert got[i] == buf[off[i]:off[i + 1]], i


def sim_msgs():
    buf = G["sim_buf"].tobytes()
    off = G["sim_off"]
    return [buf[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def sim_ref(s):
    return (int(G["sim_status"][s]), G["sim_ego"][s], G["sim_prev_x"][s], G["sim_prev_y"][s],
            int(G["sim_n_prev"][s]), G["sim_car_id"][s], G["sim_cars"][s])


def traj_dumps():
    buf, off = G["traj_buf"].tobytes(), G["traj_off"]
    return [buf[off[i]:off[i + 1]] for i in range(len(off) - 1)]


def test_sim_fixture_host_codec():
    """Simulator-shaped frames and planner-like dumps (the reference's fields and bytes in the
    fixture's sim_* / traj_* arrays): the host codec, bit and byte for byte."""
    msgs = sim_msgs()
    d, st = ppamd.telemetry_parse(msgs, car_stride=12)
    for s in range(len(msgs)):
        check_frame(d, st, s, sim_ref(s))
    got = ppamd.control_format(G["traj_x"], G["traj_y"], G["traj_n"])
    assert got == traj_dumps()


def test_format_roundtrip_through_parse():
    """Control output parsed back as the next frame's previous path recovers at least %.15g."""
    rng = np.random.default_rng(3)
    S, N = 64, 50
    xs, ys = rng.uniform(-3000, 3000, (N, S)), rng.uniform(-3000, 3000, (N, S))
    ctrl = ppamd.control_format(xs, ys, np.full(S, N, np.int32))
    frames = []
    for s in range(S):
        body = ctrl[s][len(b'42["control",'):-1]
        nx = body[body.index(b"[") + 1:body.index(b"]")]
        ny = body[body.rindex(b"[") + 1:body.rindex(b"]")]
        frames.append(b'42["telemetry",{"x":0,"y":0,"yaw":0,"speed":0,"previous_path_x":[' + nx +
                      b'],"previous_path_y":[' + ny + b'],"sensor_fusion":[]}]')
    d, st = ppamd.telemetry_parse(frames)
    assert (st == 0).all() and (d["n_prev"] == N).all()
    np.testing.assert_allclose(d["prev_x"], xs[:10], rtol=1e-14)


def test_bad_arguments():
    import ctypes as C
    off = np.zeros(2, np.int64)
    st = np.zeros(1, np.int32)
    d = ppamd.alloc_scenes(0, 12)
    b = ppamd.scene_struct(d)
    rc = ppamd.lib.pp_telemetry_parse(b"", off.ctypes.data_as(C.POINTER(C.c_int64)), 1, C.byref(b),
                                      st.ctypes.data_as(C.POINTER(C.c_int32)), 1)
    assert rc == -1                      # batch smaller than the message count


@pytest.mark.skipif(oracle_lib.load_ref_json() is None, reason="reference codec not built (no reference here)")
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_parse_and_format_vs_reference_live(seed):
    rj = oracle_lib.load_ref_json()
    msgs = codec_corpus.corpus(seed, 500)
    d, st = ppamd.telemetry_parse(msgs, car_stride=16)
    for s, m in enumerate(msgs):
        check_frame(d, st, s, oracle_lib.ref_json_parse(rj, m))
    vals = codec_corpus.control_values(seed, 200)
    rng = np.random.default_rng(seed)
    for _ in range(40):
        n = int(rng.integers(0, 60))
        x, y = rng.choice(vals, n), rng.choice(vals, n)
        got = ppamd.control_format(x[:, None], y[:, None], np.array([n], np.int32))[0]
        assert got == oracle_lib.ref_json_dump(rj, x, y)


@pytest.mark.gpu
class TestDeviceCodec:
    """The GPU codec (pp_codec.hip) against the reference's own outputs (codec_golden.npz, made by
    the reference's hasData + json.hpp) and against the host codec: same statuses (the device hands
    frames with libc-only numbers to the host: status 4), same bits, same bytes."""

    def test_parse_vs_reference_fixture(self):
        """Device-parsed fields == the reference's (src/helpers.h:15-25, src/main.cpp:1225-1252
        via json.hpp), bit for bit: the simulator-shaped frames all on the GPU, and the adversarial
        corpus's frames wherever the device does not hand them to the host."""
        msgs = sim_msgs()
        dd, ds = ppamd.telemetry_parse_device(msgs, car_stride=12)
        dd = {k: v.cpu().numpy() for k, v in dd.items()}
        ds = ds.cpu().numpy()
        assert (ds != ppamd.MSG_HOST).all()
        for s in range(len(msgs)):
            check_frame(dd, ds, s, sim_ref(s))
        msgs = golden_msgs()
        dd, ds = ppamd.telemetry_parse_device(msgs, car_stride=16)
        dd = {k: v.cpu().numpy() for k, v in dd.items()}
        ds = ds.cpu().numpy()
        on = np.flatnonzero(ds != ppamd.MSG_HOST)
        assert len(on) > 0
        for s in on:
            n = int(G["n_cars"][s])
            check_frame(dd, ds, s, (int(G["status"][s]), G["ego"][s], G["prev_x"][s], G["prev_y"][s],
                                    int(G["n_prev"][s]), G["car_id"][s][:n], G["cars"][s][:n]))

    def test_format_vs_reference_fixture(self):
        """Device-formatted control messages == the reference's msgJson.dump() bytes
        (src/main.cpp:1461-1466, json.hpp:6689-6692 %.15g): planner-like values all on the GPU."""
        import torch
        dev = torch.device("cuda", 0)
        slots, ln = ppamd.control_format_device(torch.from_numpy(G["traj_x"]).to(dev),
                                                torch.from_numpy(G["traj_y"]).to(dev),
                                                torch.from_numpy(G["traj_n"]).to(dev))
        got = ppamd.slots_to_messages(slots, ln)
        assert got == traj_dumps()

    def compare_parse(self, msgs):
        hd, hs = ppamd.telemetry_parse(msgs, car_stride=16)
        dd, ds = ppamd.telemetry_parse_device(msgs, car_stride=16)
        dd = {k: v.cpu().numpy() for k, v in dd.items()}
        ds = ds.cpu().numpy()
        host = ds == ppamd.MSG_HOST
        assert ((ds == hs) | (host & np.isin(hs, [0, 2]))).all()
        ok = ~host & np.isin(hs, [0, 2])
        for k in hd:
            a, b = np.asarray(hd[k])[..., ok], dd[k][..., ok]
            if a.dtype.kind == "f":
                assert (a.view(np.uint64) == b.view(np.uint64)).all(), k
            else:
                assert (a == b).all(), k
        return int(ok.sum()), int(host.sum())

    def test_parse_golden_and_random(self):
        # adversarial spellings: most frames hold some >19-digit number and go to the host codec
        n_ok, n_host = self.compare_parse(golden_msgs())
        assert n_ok > 0 and n_host > 0
        for seed in (31, 32):
            self.compare_parse(codec_corpus.corpus(seed, 3000))

    def test_parse_simulator_like_frames_on_device(self):
        """Frames as a simulator writes them (shortest round-trip numbers): all parsed on the GPU."""
        import sys
        import os
        sys.path.insert(0, os.path.join(oracle_lib.REPO, "tools"))
        from bench_serving import frames_from_scenes
        m = ppamd.Map(*oracle_lib.highway_map())
        msgs = frames_from_scenes(ppamd.synth_host(m, 2000, seed=9))
        n_ok, n_host = self.compare_parse(msgs)
        assert n_ok == 2000 and n_host == 0

    def test_parse_many_rows_on_device(self):
        """Frames with up to 250 sensor_fusion rows (duplicate and negative ids included) parse on
        the GPU with a 256-column batch, bit for bit the host codec's std::map order; a frame with
        more rows than the batch's columns goes to the host (status 4)."""
        rng = np.random.default_rng(17)
        msgs = []
        for k, n in enumerate([0, 12, 24, 25, 40, 100, 180, 250, 256, 300]):
            ids = rng.integers(-50, 400, n)
            rows = ",".join("[%d,%r,%r,%r,%r,0,0]" % (int(i), float(rng.uniform(0, 3000)), float(rng.uniform(0, 3000)),
                                                      float(rng.normal(0, 10)), float(rng.normal(0, 10)))
                            for i in ids)
            msgs.append(('42["telemetry",{"x":%r,"y":%r,"yaw":%r,"speed":%r,"previous_path_x":[1.5,2.5],'
                         '"previous_path_y":[3.5,4.5],"sensor_fusion":[%s]}]'
                         % (float(rng.uniform(0, 3000)), float(rng.uniform(0, 3000)), 12.5, 30.25, rows)).encode())
        hd, hs = ppamd.telemetry_parse(msgs, car_stride=256)
        dd, ds = ppamd.telemetry_parse_device(msgs, car_stride=256)
        dd = {k: v.cpu().numpy() for k, v in dd.items()}
        ds = ds.cpu().numpy()
        # raw rows beyond the 256 columns: the device hands the frame to the host
        assert ds[-1] == ppamd.MSG_HOST and ds[-2] in (0, ppamd.MSG_HOST)
        on = ds != ppamd.MSG_HOST
        assert on[:8].all() and (ds[on] == hs[on]).all()
        assert hd["n_cars"][on].max() > 64
        for k in hd:
            a, b = np.asarray(hd[k])[..., on], dd[k][..., on]
            if a.dtype.kind == "f":
                assert (a.view(np.uint64) == b.view(np.uint64)).all(), k
            else:
                assert (a == b).all(), k

    def format_both(self, xs, ys, n_out):
        import torch
        want = ppamd.control_format(xs, ys, n_out)
        dev = torch.device("cuda", 0)
        slots, ln = ppamd.control_format_device(torch.from_numpy(xs).to(dev), torch.from_numpy(ys).to(dev),
                                                torch.from_numpy(n_out).to(dev))
        got = ppamd.slots_to_messages(slots, ln)
        n_dev = 0
        for s in range(len(want)):
            if got[s] is not None:
                assert got[s] == want[s], s
                n_dev += 1
        return n_dev

    def test_format_matches_host(self):
        rng = np.random.default_rng(5)
        S, N = 4096, 50
        # adversarial values (many outside fmt15g's domain -> host): identical wherever formatted
        vals = codec_corpus.control_values(5, 3000)
        n_dev = self.format_both(rng.choice(vals, (N, S)), rng.choice(vals, (N, S)),
                                 rng.integers(0, N + 1, S).astype(np.int32))
        assert n_dev > 0
        # trajectories as the planner writes them: every message on the GPU
        xs = rng.uniform(-3000, 3000, (N, S)) * 10.0 ** rng.integers(-3, 4, (N, S))
        xs[::7] = np.round(xs[::7])
        xs[::11] = np.nan
        ys = rng.uniform(-3000, 3000, (N, S))
        assert self.format_both(xs, ys, rng.integers(0, N + 1, S).astype(np.int32)) == S

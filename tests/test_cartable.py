"""Sensor-fusion car tables of any size and any int ids (the reference's std::map<int, Car>
sensor_fusion_cars, src/main.cpp:1194, 1325-1350, and its id -1 "no car" sentinel at :1383-1432).

- CPU: the C restatement equals the reference's own code on frames with 24 rows and ids that are
  negative (-1 included), sparse and large.
- GPU: pp_eval with 24 rows against the restatement; pp_plan_frame (the host std::map laid out as
  table slots over the union of the stored and reported ids, csrc/pp_cartable.h) driven through
  closed-loop episodes next to a reference session that keeps the real std::map — 24 cars with ids
  >= 16, a sensor range that leaves stale entries, cars dropping out of the road (erased), and ids
  that include -1."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd


def many_car_scenes(m, S, seed, ids_fn, rows=24):
    """S synthetic scenes with `rows` sensor_fusion rows: the cars of ceil(rows / 12) generator
    batches side by side, rows reordered by the ids ids_fn(rng, rows) (ascending, as the batch
    contract requires); every 7th scene reports 5 rows fewer."""
    bs = [ppamd.synth_host(m, S, seed=seed + i, first=0) for i in range((rows + 11) // 12)]
    sc = {k: v for k, v in bs[0].items()}
    for k in ("car_x", "car_y", "car_vx", "car_vy"):
        sc[k] = np.ascontiguousarray(np.concatenate([b[k] for b in bs], 0)[:rows])
    rng = np.random.default_rng(seed)
    ids = np.zeros((rows, S), np.int32)
    for s in range(S):
        ids[:, s] = np.sort(ids_fn(rng, rows))
    sc["car_id"] = ids
    sc["n_cars"] = np.full(S, rows, np.int32)
    sc["n_cars"][::7] = rows - 5
    return sc


def ids_wide(rng, n):
    """distinct ascending ints: negatives (-1 in about half the scenes), sparse, up to 2^30"""
    pool = np.concatenate([rng.choice(np.arange(-40, 0), 3, replace=False),
                           rng.choice(np.arange(16, 2 ** 30, 9973), n, replace=False)])
    if rng.random() < 0.5:
        pool[0] = -1
    return rng.choice(np.unique(pool), n, replace=False)


@pytest.mark.parametrize("rows", [24, ppamd.MAX_CARS])
def test_restatement_equals_reference_many_cars(rows):
    rlib = oracle_lib.load_ref()
    olib = oracle_lib.load_oracle()
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    sc = many_car_scenes(m, 600 if rows <= 24 else 200, 4711, ids_wide, rows)
    prm = ppamd.default_params(n_speeds=5)
    ref = oracle_lib.ref_eval(rlib, wx, wy, sc, 5, [prm.speed_offsets[i] for i in range(4)])
    got = oracle_lib.oracle_eval(olib, wx, wy, sc, ppamd.default_params(n_speeds=5, emit_paths=True), info=True)
    assert np.array_equal(np.stack([got["next_x"].T, got["next_y"].T], -1), ref["ref_next"])
    assert np.array_equal(got["n_out"], ref["ref_n"])
    gp = np.transpose(got["paths"], (0, 2, 1, 3))
    assert np.array_equal(np.nan_to_num(gp, nan=7e7), np.nan_to_num(ref["paths"], nan=7e7))
    # the -1 sentinel matters on some scenes: a car with id -1 was the nearest in-lane car
    assert (got["info"]["in_lane_car"] == -1).sum() > 0


# ---- closed-loop episodes through pp_plan_frame -------------------------------------------------
class Traffic:
    """Cars following lane centre polylines (map geometry), seeded; ids given."""

    def __init__(self, geom, ids, rng, ego_s0):
        self.lc = [geom[:, 4 + 2 * L:6 + 2 * L] for L in range(ppamd.NUM_LANES)]
        seg = [np.hypot(*np.diff(np.vstack([c, c[:1]]), axis=0).T) for c in self.lc]
        self.cum = [np.concatenate([[0], np.cumsum(s)]) for s in seg]
        self.ids = list(ids)
        n = len(ids)
        self.lane = rng.integers(0, ppamd.NUM_LANES, n)
        self.s = (ego_s0 + rng.uniform(-60, 260, n)) % self.cum[0][-1]
        self.v = rng.uniform(4, 26, n)
        self.off = rng.uniform(-0.4, 0.4, n)
        self.leave = rng.random(n) < 0.25           # leave the road after frame 40 (matching fails > 1 km off)

    def pos(self, j):
        L = self.lane[j]
        c, cum = self.lc[L], self.cum[L]
        s = self.s[j] % cum[-1]
        i = int(np.searchsorted(cum, s, side="right") - 1)
        a, b = c[i % len(c)], c[(i + 1) % len(c)]
        t = (s - cum[i]) / (cum[i + 1] - cum[i])
        u = (b - a) / np.hypot(*(b - a))
        p = a + t * (b - a) + self.off[j] * np.array([u[1], -u[0]])
        return p, u * self.v[j]

    def step(self, dt, f):
        self.s += self.v * dt
        self.off = np.where(self.leave & (f > 40), self.off + 60.0, self.off)


def run_episode(env, ids, frames, seed, sensor_range):
    m, wx, wy = env["m"], env["wx"], env["wy"]
    rlib = env["rlib"]
    geom = m.geometry()
    rng = np.random.default_rng(seed)
    # ego starts on a lane centre with a previous path along it
    sc = ppamd.synth_host(m, 1, seed=seed, first=0)
    ego = [float(sc["ego_x"][0]), float(sc["ego_y"][0]), float(sc["ego_yaw_deg"][0]), float(sc["ego_speed_mph"][0])]
    prev = np.stack([sc["prev_x"][:, 0], sc["prev_y"][:, 0]], 1)
    n_prev = int(sc["n_prev"][0])
    traffic = Traffic(geom, ids, rng, 0.0)
    # place the traffic near the ego: shift each car's s so it starts within the sensor window
    ego_pt = np.array(ego[:2])
    for j in range(len(ids)):
        c, cum = traffic.lc[traffic.lane[j]], traffic.cum[traffic.lane[j]]
        k = int(np.argmin(np.hypot(*(c - ego_pt).T)))
        traffic.s[j] = (cum[k] + rng.uniform(-50, 200)) % cum[-1]
    ppamd.plan_reset(m)
    h = rlib.ref_session_new(oracle_lib._arr(wx), oracle_lib._arr(wy), len(wx), 1)
    tl_gpu = 1
    worst, stale, erased, reported_max = 0.0, 0, 0, 0
    try:
        for f in range(frames):
            rows = []
            for j, cid in enumerate(traffic.ids):
                p, v = traffic.pos(j)
                if np.hypot(*(p - np.array(ego[:2]))) <= sensor_range:
                    rows.append((cid, p[0], p[1], v[0], v[1]))
            reported_max = max(reported_max, len(rows))
            # reference session (one scene, rows in any order: the reference iterates them as sent)
            order = rng.permutation(len(rows))
            rows_sent = [rows[i] for i in order]
            one = oracle_lib.one_scene(ego, prev[:n_prev], rows_sent, tl_gpu)
            nxy = np.zeros(100)
            n_out = C.c_int()
            tl_ref = C.c_int()
            ntab = C.c_int()
            rlib.ref_session_frame(h, C.byref(one["struct"]), nxy.ctypes.data_as(oracle_lib._dp), C.byref(n_out),
                                   C.byref(tl_ref), C.byref(ntab))
            nx, ny, tl_gpu = ppamd.plan_frame(m, ego[0], ego[1], ego[2], ego[3], prev[:n_prev, 0], prev[:n_prev, 1],
                                              rows_sent, target_lane=tl_gpu)
            n = n_out.value
            assert len(nx) == n and tl_gpu == tl_ref.value, (f, len(nx), n, tl_gpu, tl_ref.value)
            ref_xy = nxy[:2 * n].reshape(n, 2)
            if n:
                worst = max(worst, float(np.abs(np.stack([nx, ny], 1) - ref_xy).max()))
            assert worst <= oracle_lib.TOL, (f, worst)
            stale += ntab.value > len(rows)
            erased += ntab.value < len(rows)
            # drive 3 points of the plan
            plan = ref_xy
            k = min(3, n)
            if k >= 1:
                q = plan[k - 2] if k >= 2 else np.array(ego[:2])
                d = plan[k - 1] - q
                ego = [plan[k - 1][0], plan[k - 1][1],
                       float(np.degrees(np.arctan2(d[1], d[0]))) if np.hypot(*d) > 0 else ego[2],
                       float(np.hypot(*d) * 50 * 2.237)]
            prev = plan[k:]
            n_prev = len(prev)
            traffic.step(0.02 * max(k, 1), f)
    finally:
        rlib.ref_session_free(h)
    return worst, stale, erased, reported_max


@pytest.mark.gpu
class TestCarTableGPU:
    @pytest.fixture(scope="class")
    def env(self):
        import torch
        wx, wy = oracle_lib.highway_map()
        return {"torch": torch, "m": ppamd.Map(wx, wy), "wx": wx, "wy": wy, "dev": torch.device("cuda", 0),
                "olib": oracle_lib.load_oracle(), "rlib": oracle_lib.load_ref_session()}

    @pytest.mark.parametrize("rows", [24, ppamd.MAX_CARS])
    def test_eval_many_cars_vs_oracle(self, env, rows):
        S = 1500 if rows <= 24 else 600
        sc = many_car_scenes(env["m"], S, 99, ids_wide, rows)
        for mode in (ppamd.COST_REFERENCE, ppamd.COST_COMFORT):
            prm = ppamd.default_params(emit_paths=True, cost_mode=mode)
            d = {k: env["torch"].from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
            r = ppamd.alloc_result(S, prm, xp="torch", device=env["dev"])
            ppamd.evaluate(env["m"], d, prm, r, device=0)
            env["torch"].cuda.synchronize()
            got = ppamd.result_to_numpy(r)
            ref = oracle_lib.oracle_eval(env["olib"], env["wx"], env["wy"], sc, prm, info=False)
            oracle_lib.compare(got, ref)

    def test_eval_rejects_more_rows_than_max(self, env):
        """car_stride > PP_MAX_CARS: PP_ERR_ARG before any launch (include/pp.h), never a truncation"""
        sc = many_car_scenes(env["m"], 64, 5, ids_wide, ppamd.MAX_CARS + 1)
        prm = ppamd.default_params()
        d = {k: env["torch"].from_numpy(np.ascontiguousarray(v)).to(env["dev"]) for k, v in sc.items()}
        r = ppamd.alloc_result(64, prm, xp="torch", device=env["dev"])
        with pytest.raises(ppamd.PPError):
            ppamd.evaluate(env["m"], d, prm, r, device=0)

    @pytest.mark.parametrize("ids,sensor_range,seed,need", [
        (list(range(1000, 1000 + 7 * 24, 7)), 60.0, 3, "stale"),   # 24 cars, ids >= 16, stale entries
        (sorted([-1, -9, 5, 17, 64, 99999, 2 ** 31 - 2, 12, 300, 301, 40, 41]), 1e5, 5, "erased"),
        (list(range(16, 40)), 45.0, 8, "stale"),
        # 100 cars with sparse ids up to 2^31 - 2 (beyond the former 64-car limit)
        (sorted(set([-(2 ** 31), -5, 0, 2 ** 31 - 2] + [int(v) for v in
                    np.random.default_rng(77).choice(2 ** 31 - 3, 96, replace=False)])), 1e5, 9, "erased"),
    ])
    def test_plan_frame_episode_vs_reference(self, env, ids, sensor_range, seed, need):
        worst, stale, erased, rep = run_episode(env, ids, 300, seed, sensor_range)
        print(f"ids {ids[:3]}..: max |dxy| {worst:.3e} m, frames with stale entries {stale}, "
              f"with erased {erased}, max reported {rep}")
        assert (stale if need == "stale" else erased) > 0

    @pytest.mark.parametrize("shape", [ppamd.SHAPE_SPLIT, ppamd.SHAPE_CAND_SMALL, ppamd.SHAPE_STEP])
    def test_plan_frame_episode_other_shapes(self, env, shape):
        """pp_plan_frame under a forced launch shape: the split and cand_small shapes leave the
        one-launch frame kernel (k_plan_frame) for its fallback, copies + pp_eval; every shape
        must give the reference's frames (30 cars, ids >= 16, stale entries)."""
        with ppamd.debug(ppamd.DBG_SHAPE, shape):
            worst, stale, erased, rep = run_episode(env, list(range(16, 46)), 80, 12, 1e5)
        assert rep > 25                                  # beyond the kernel-argument inputs too


@pytest.mark.gpu
@pytest.mark.parametrize("S", [37, 5000])
def test_table_padding_with_int32_max_car_id(S):
    """pp_cartable.h pads a scene's slots past its union with id INT32_MAX; a real car may carry
    that id too. With an empty table and every car reported, the frame must equal the table-free
    evaluation for every K1 group size: the padding slots repeat the last id and match no row."""
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    dev = torch.device("cuda", 0)
    host = ppamd.synth_host(m, S, seed=616, first=5_000_000)
    host["car_id"][11] = np.int32(2 ** 31 - 1)
    prm = ppamd.default_params(emit_paths=True)

    def run(d):
        dd = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
        rr = ppamd.alloc_result(S, prm, xp="torch", device=dev)
        ppamd.evaluate(m, dd, prm, rr, device=0)
        torch.cuda.synchronize()
        return ppamd.result_to_numpy(rr), {k: dd[k].cpu().numpy() for k in dd}

    base, _ = run(host)
    sc = ppamd.add_car_table(dict(host), slots=16)
    sc["tab_id"][:12] = host["car_id"]
    sc["tab_id"][12:] = 2 ** 31 - 1                     # padding: INT32_MAX, empty
    try:
        for G in (1, 2, 4, 8, 16):
            ppamd.set_prep_group(G)
            got, st = run(sc)
            for k, v in base.items():
                assert np.array_equal(np.ascontiguousarray(v).view(np.uint8),
                                      np.ascontiguousarray(got[k]).view(np.uint8)), (G, k)
            assert (st["tab_valid"][12:] == 0).all(), G
    finally:
        ppamd.set_prep_group(0)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 37, 600, 5000])
def test_table_mode_group_invariance(S):
    """Car-table mode through K1 with G = 1 (one lane per scene) and G = 2..16 (the grouped K1: slots
    split over the group, planner in slot order): the same outputs and the same updated table, bit
    for bit. The table state has reported, stale and erased slots: a first frame fills it, the
    second reports only some of the cars (the others stay as stale slots)."""
    import torch
    wx, wy = oracle_lib.highway_map()
    m = ppamd.Map(wx, wy)
    dev = torch.device("cuda", 0)
    host = ppamd.synth_host(m, S, seed=515, first=3_000_000)
    prm = ppamd.default_params(emit_paths=True)

    def to_dev(d):
        return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}

    sc = ppamd.add_car_table(dict(host), slots=12)
    d0 = to_dev(sc)
    r = ppamd.alloc_result(S, prm, xp="torch", device=dev)
    ppamd.set_prep_group(1)
    try:
        ppamd.evaluate(m, d0, prm, r, device=0)          # frame 1 fills the table
        torch.cuda.synchronize()
        state = {k: v.cpu().numpy() for k, v in d0.items()}
        rng = np.random.default_rng(S)
        state["n_cars"] = rng.integers(0, 13, S).astype(np.int32)   # frame 2 reports a prefix of the rows
        outs = {}
        for G in (1, 2, 4, 8, 16):
            ppamd.set_prep_group(G)
            d = to_dev(state)
            rr = ppamd.alloc_result(S, prm, xp="torch", device=dev)
            ppamd.evaluate(m, d, prm, rr, device=0)
            torch.cuda.synchronize()
            outs[G] = ({k: v for k, v in ppamd.result_to_numpy(rr).items()},
                       {k: d[k].cpu().numpy() for k in ppamd.TABLE_FIELDS_I + ppamd.TABLE_FIELDS_F})
    finally:
        ppamd.set_prep_group(0)
    assert (state["tab_valid"].sum(0) > state["n_cars"]).any()      # stale slots present
    for G in (2, 4, 8, 16):
        for k, v in outs[1][0].items():
            assert np.array_equal(np.ascontiguousarray(v).view(np.uint8), np.ascontiguousarray(outs[G][0][k]).view(np.uint8)), (G, k)
        for k, v in outs[1][1].items():
            assert np.array_equal(v.view(np.uint8), outs[G][1][k].view(np.uint8)), (G, k)

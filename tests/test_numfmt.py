"""Exactness of the codec's integer number conversions (csrc/pp_numfmt.h) — checked through
pp_telemetry_parse / pp_control_format against Python's correctly rounded float() and '%.15g'
(the same results as glibc's strtod / snprintf that nlohmann calls): ties, carries, decade
edges, the fast-path domain boundaries and the libc fallbacks."""
import numpy as np

from oracle_lib import ppamd


def dump(v):
    if not np.isfinite(v):
        return "null"
    t = "%.15g" % v
    return t + ("" if ("." in t or "e" in t) else ".0")


def hard_doubles(rng, n):
    parts = [
        rng.uniform(-5000, 5000, n),
        rng.standard_normal(n) * 10.0 ** rng.integers(-16, 20, n),
        np.round(rng.uniform(-1e15, 1e15, n)) + 0.5,                 # 16-digit ties
        (rng.integers(10 ** 14, 10 ** 15, n).astype(np.float64) + 0.5) * 10.0 ** rng.integers(-10, 3, n),
        np.nextafter(10.0 ** rng.integers(-14, 19, n), np.inf * rng.choice([-1, 1], n)),
        10.0 ** rng.integers(-14, 19, n),
        1e15 - rng.uniform(0, 1, n), 1e18 * rng.uniform(0.9, 1.1, n), 1e-13 * rng.uniform(0.9, 1.1, n),
        np.round(rng.uniform(-1e6, 1e6, n)),
        rng.uniform(0, 1, n) * 2.0 ** rng.integers(-60, 70, n),
    ]
    v = np.concatenate(parts)
    return v[np.isfinite(v)]


def test_format_matches_correctly_rounded_g15():
    rng = np.random.default_rng(1)
    v = hard_doubles(rng, 4000)
    v = np.concatenate([v, [0.0, -0.0, np.nan, np.inf, -np.inf, 5e-324, 1.7976931348623157e308,
                            999999999999999.4, 999999999999999.5, 99999999999999.95, 0.0001, 9.99999999999999e-5]])
    N = 50
    S = len(v) // N
    xs = v[:N * S].reshape(S, N).T.copy()       # [N][S]
    ys = xs[::-1].copy()
    got = ppamd.control_format(xs, ys, np.full(S, N, np.int32))
    for s in range(S):
        want = ('42["control",{"next_x":[' + ",".join(dump(x) for x in xs[:, s]) + '],"next_y":[' +
                ",".join(dump(y) for y in ys[:, s]) + "]}]").encode()
        assert got[s] == want, (s, got[s][:200], want[:200])


def number_strings(rng, n):
    out = []
    for v in hard_doubles(rng, n // 10):
        k = rng.integers(0, 6)
        out.append(repr(float(v)) if k == 0 else ("%.17g" % v) if k == 1 else ("%.20e" % v) if k == 2
                   else ("%.15g" % v) if k == 3 else ("%.3f" % v) if k == 4 else ("%.25g" % v))
    for _ in range(n // 4):                    # random decimal literals, 1..26 digits, exponents
        nd = int(rng.integers(1, 27))
        digits = "".join(str(int(d)) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        t = (digits[:dot] or "0") + ("." + digits[dot:] if dot < nd else "")
        t = t.lstrip("0") or "0"
        if t.startswith("."):
            t = "0" + t
        if rng.random() < 0.5:
            t += "e%d" % int(rng.integers(-40, 40))
        if rng.random() < 0.5:
            t = "-" + t
        out.append(t)
    return [s.replace("inf", "1e400").replace("nan", "0") for s in out]


def test_parse_matches_correctly_rounded_float():
    rng = np.random.default_rng(2)
    nums = number_strings(rng, 20000)
    nums += ["0", "-0", "-0.0", "18446744073709551615", "18446744073709551616", "-9223372036854775808",
             "-9223372036854775809", "9007199254740993", "1e-27", "1e27", "1e28", "1e-28",
             "9999999999999999999", "12345678901234567890123e-5", "4.9e-324", "1.7976931348623157e308"]
    per = 74
    msgs, exp = [], []
    for i in range(0, len(nums), per):
        chunk = nums[i:i + per] + ["1"] * (per - len(nums[i:i + per]))
        px, py, cars = chunk[:5], chunk[5:10], chunk[10:]
        rows = ",".join("[%d,%s,%s,%s,%s,0,0]" % (j, *cars[4 * j:4 * j + 4]) for j in range(16))
        msgs.append(('42["telemetry",{"x":1,"y":2,"yaw":3,"speed":4,"previous_path_x":[%s],'
                     '"previous_path_y":[%s],"sensor_fusion":[%s]}]' % (",".join(px), ",".join(py), rows)).encode())
        exp.append(chunk)
    d, st = ppamd.telemetry_parse(msgs, car_stride=16)
    assert (st == 0).all()
    for s, chunk in enumerate(exp):
        want = np.array([float(t) for t in chunk])
        got = np.concatenate([d["prev_x"][:5, s], d["prev_y"][:5, s],
                              np.stack([d["car_x"][:, s], d["car_y"][:, s], d["car_vx"][:, s], d["car_vy"][:, s]], 1).ravel()])
        bad = got.view(np.uint64) != want.view(np.uint64)
        # nlohmann's integer tokens: "-0" -> +0.0 (strtoll), the only deviation from float()
        for i in np.nonzero(bad)[0]:
            assert chunk[i] in ("-0",), (chunk[i], got[i], want[i])

"""Telemetry / control corpora for the wire-codec parity tests (tests/test_codec.py).

Frames follow the simulator's format (`42["telemetry",{"x":..,"y":..,"yaw":..,"speed":..,"s":..,
"d":..,"previous_path_x":[..],"previous_path_y":[..],"end_path_s":..,"end_path_d":..,
"sensor_fusion":[[id,x,y,vx,vy,s,d],..]}]`) with the number spellings a JSON writer may produce
(shortest round-trip, %.15g, fixed, integers, exponents, signed zeros, 20-digit integers, long
mantissas), whitespace, shuffled / duplicated / fractional car ids, plus non-telemetry frames
(manual `null`, other events, truncated or malformed ones)."""
import numpy as np


def spell(rng, v):
    k = rng.integers(0, 12)
    if k == 0:
        return repr(float(v))
    if k == 1:
        return "%.15g" % v
    if k == 2:
        return "%.6f" % v
    if k == 3:
        return "%.17g" % v
    if k == 4:
        return "%.3e" % v
    if k == 5:
        return str(int(v))
    if k == 6:
        return "%.25f" % v
    if k == 7:
        return "%.10E" % v
    if k == 8:
        return ("%.15g" % v).replace("e-0", "e-").replace("e+0", "e")
    if k == 9:
        return "%.0f" % v
    if k == 10:
        return "%.1f" % v
    return repr(float(v))


SPECIAL = ["0", "-0", "-0.0", "0.0", "1e-05", "1E+2", "-1e-320", "4.9e-324", "2.2250738585072014e-308",
           "1.7976931348623157e308", "18446744073709551615", "18446744073709551616", "-9223372036854775808",
           "-9223372036854775809", "123456789012345678901", "9007199254740993", "0.1000000000000000055511151231257827",
           "3.14159265358979323846264338327950288", "1e22", "1e23", "7.8e-5", "123456.789e3", "0.000000000000000000000123"]


def telemetry(rng, n_prev, n_cars, ws=False, dup=False, frac_id=False, special=False):
    sp = (lambda v: SPECIAL[rng.integers(0, len(SPECIAL))] if special and rng.random() < 0.3 else spell(rng, v))
    sep = (lambda: " " * int(rng.integers(0, 3)) + ("\n" if rng.random() < 0.1 else "")) if ws else (lambda: "")
    x, y = rng.uniform(-3000, 3000), rng.uniform(-3000, 3000)
    px = x + np.cumsum(rng.uniform(0, 0.5, n_prev))
    py = y + np.cumsum(rng.uniform(-0.1, 0.1, n_prev))
    ids = list(range(n_cars))
    rng.shuffle(ids)
    if dup and n_cars > 2:
        ids[1] = ids[0]
    rows = []
    for i in ids:
        cid = ("%d.%d" % (i, rng.integers(0, 10))) if frac_id else str(i)
        vals = [rng.uniform(-3000, 3000), rng.uniform(-3000, 3000), rng.uniform(-30, 30), rng.uniform(-30, 30),
                rng.uniform(0, 7000), rng.uniform(-2, 14)]
        rows.append("[" + sep() + cid + "," + ",".join(sep() + sp(v) for v in vals) + "]")
    obj = ('{"x":' + sep() + sp(x) + ',"y":' + sp(y) + ',"yaw":' + sp(rng.uniform(-360, 360)) +
           ',"speed":' + sp(rng.uniform(0, 50)) + ',"s":' + sp(rng.uniform(0, 7000)) + ',"d":' + sp(rng.uniform(0, 12)) +
           ',"previous_path_x":[' + ",".join(sp(v) for v in px) + '],"previous_path_y":[' +
           ",".join(sp(v) for v in py) + '],"end_path_s":' + sp(1.0) + ',"end_path_d":' + sp(2.0) +
           ',"sensor_fusion":[' + ",".join(rows) + "]}")
    return ("42[" + sep() + '"telemetry",' + sep() + obj + "]").encode()


def corpus(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for m in range(n):
        kind = m % 10
        if kind == 7:
            out.append(rng.choice([b'42["telemetry",null]', b'42["manual",{}]', b'42["other",{"x":1}]', b"2",
                                   b"43[]", b'42["telemetry",{"x":1,"y":2}]', b'42["telemetry",{"x":1,',
                                   b'42["telemetry",{"x":1,"y":2,"yaw":3,"speed":4,"previous_path_x":[1],'
                                   b'"previous_path_y":[],"sensor_fusion":[]}]',
                                   b'42["telemetry",{"x":1e,"y":2}]']))
            continue
        n_prev = int(rng.choice([0, 3, 10, 11, 47]))
        out.append(telemetry(rng, n_prev, int(rng.integers(0, 15)), ws=kind == 1, dup=kind == 2,
                             frac_id=kind == 3, special=kind in (4, 5)))
    return out


def control_values(seed, n):
    rng = np.random.default_rng(seed)
    v = np.concatenate([rng.uniform(-3000, 3000, n), rng.normal(0, 1, n) * 10.0 ** rng.integers(-30, 30, n),
                        np.round(rng.uniform(-1000, 1000, n)), [0.0, -0.0, np.nan, np.inf, -np.inf, 1e15, 1e16,
                                                                 123456789012345.0, 5e-324, 1.7976931348623157e308, 0.1]])
    return v


def sim_spell(rng, v):
    """The spellings a simulator-side JSON writer produces (at most 17 significant digits)."""
    k = rng.integers(0, 5)
    if k == 0:
        return "%.15g" % v
    if k == 1:
        return "%.17g" % v
    if k == 2:
        return "%.6f" % v
    if k == 3 and abs(v) < 1e6:
        return str(int(v))
    return repr(float(v))


def sim_corpus(seed, n):
    """Simulator-shaped telemetry: every number within the device codec's exact domain (so the GPU
    parses every frame itself), 12 cars, 0-47 previous points, a manual frame every 16th."""
    rng = np.random.default_rng(seed)
    out = []
    for m in range(n):
        if m % 16 == 15:
            out.append(b'42["telemetry",null]' if m % 32 == 15 else b'42["manual",{}]')
            continue
        sp = lambda v: sim_spell(rng, v)
        n_prev = int(rng.choice([0, 10, 47]))
        x, y = rng.uniform(0, 3000), rng.uniform(0, 3000)
        px = x + np.cumsum(rng.uniform(0, 0.45, n_prev))
        py = y + np.cumsum(rng.uniform(-0.05, 0.05, n_prev))
        rows = ",".join("[%d,%s,%s,%s,%s,%s,%s]" % (j, sp(rng.uniform(0, 3000)), sp(rng.uniform(0, 3000)),
                                                    sp(rng.uniform(-25, 25)), sp(rng.uniform(-25, 25)),
                                                    sp(rng.uniform(0, 7000)), sp(rng.uniform(0, 12)))
                        for j in range(12))
        out.append(('42["telemetry",{"x":%s,"y":%s,"yaw":%s,"speed":%s,"s":%s,"d":%s,"previous_path_x":[%s],'
                    '"previous_path_y":[%s],"end_path_s":%s,"end_path_d":%s,"sensor_fusion":[%s]}]'
                    % (sp(x), sp(y), sp(rng.uniform(0, 360)), sp(rng.uniform(0, 50)), sp(rng.uniform(0, 7000)),
                       sp(rng.uniform(0, 12)), ",".join(sp(v) for v in px), ",".join(sp(v) for v in py),
                       sp(rng.uniform(0, 7000)), sp(rng.uniform(0, 12)), rows)).encode())
    return out


def trajectory_values(seed, N, S):
    """Planner-like next_x/next_y (point-major [N][S]): magnitudes 1e-3..1e6, some integral values,
    some NaN (the control dump's `null`)."""
    rng = np.random.default_rng(seed)
    xs = rng.uniform(-3000, 3000, (N, S)) * 10.0 ** rng.integers(-3, 4, (N, S))
    xs[::7] = np.round(xs[::7])
    xs[::11, ::3] = np.nan
    ys = rng.uniform(-3000, 3000, (N, S))
    n_out = rng.integers(0, N + 1, S).astype(np.int32)
    n_out[:4] = (0, 1, N, N)
    return xs, ys, n_out

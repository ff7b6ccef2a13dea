"""The reference's libm restated (csrc/pp_glibcm.h): glibc 2.35's x86-64 sin, cos and atan2 bit
for bit, host build and device build. The frame's heading and its rotations (src/main.cpp:607,
786-787, 822-823) come from it, so every knot, path point and the standstill 0/0 branch
(src/main.cpp:1025) carry the reference's exact bits."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ppamd

REPO = oracle_lib.REPO


def args(n, seed):
    """Headings, degree conversions, small and medium angles, step vectors of all lengths."""
    rng = np.random.default_rng(seed)
    x = np.concatenate([rng.uniform(-np.pi, np.pi, n), rng.uniform(-1440, 1440, n) * np.pi / 180,
                        rng.uniform(-1, 1, n) * 2.0 ** -rng.integers(0, 60, n),
                        rng.uniform(-1, 1, n) * 2.0 ** rng.integers(0, 26, n),
                        [0.0, -0.0, 5e-324, 1e-310, 0.126, 0.855469, 2.426265, np.inf, np.nan]])
    th = rng.uniform(-np.pi, np.pi, 2 * n)
    ln = 2.0 ** rng.uniform(-16, 8, 2 * n)
    y2, x2 = ln * np.sin(th), ln * np.cos(th)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 5e-324, 1e300])
    ys, xs = np.meshgrid(sp, sp)
    wide_y = rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-1000, 1000, n)
    wide_x = rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-1000, 1000, n)
    return x, np.concatenate([y2, ys.ravel(), wide_y]), np.concatenate([x2, xs.ravel(), wide_x])


def same(a, b):
    """Bit for bit (signed zeros included: atan2 and the standstill branch are sign sensitive);
    NaNs match any NaN payload."""
    a, b = np.ascontiguousarray(a, np.float64), np.ascontiguousarray(b, np.float64)
    return bool(((a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))).all())


def test_oracle_builds_call_sin_and_cos_separately():
    """The reference's -O0 build calls sin and cos; the oracle builds must not let GCC fuse a
    sin/cos pair into glibc's sincos (different results in ~0.05 % of arguments)."""
    for so in ("oracle/liboracle.so", "oracle/_ref/libppref.so"):
        p = os.path.join(REPO, so)
        if not os.path.exists(p):
            continue
        syms = subprocess.run(["nm", "-D", p], capture_output=True, text=True, check=True).stdout
        assert " sincos" not in syms, so


def test_host_build_equals_glibc():
    olib = oracle_lib.load_oracle()
    x, y, z = args(200_000, 1)
    for k in ("sin", "cos"):
        got = ppamd.libm_eval(k, x)
        ref = oracle_lib.glibc_batch(olib, k, x)
        assert same(got, ref), (k, x[got != ref][:4])
    got = ppamd.libm_eval("atan2", y, z)
    ref = oracle_lib.glibc_batch(olib, "atan2", y, z)
    assert same(got, ref), (y[got != ref][:4], z[got != ref][:4])


def test_standalone_checker():
    """tools/glibcm_check.cpp: 2 x 10^6 further arguments per function, compiled here."""
    exe = "/tmp/pp_glibcm_check"
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", "-fno-builtin-sin", "-fno-builtin-cos",
                    os.path.join(REPO, "tools", "glibcm_check.cpp"), "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe, "1000000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]


@pytest.mark.gpu
def test_device_build_equals_glibc():
    import torch
    olib = oracle_lib.load_oracle()
    dev = torch.device("cuda", 0)
    x, y, z = args(400_000, 2)
    for k in ("sin", "cos"):
        got = ppamd.libm_eval(k, torch.from_numpy(x).to(dev), device=0).cpu().numpy()
        assert same(got, oracle_lib.glibc_batch(olib, k, x)), k
    got = ppamd.libm_eval("atan2", torch.from_numpy(y).to(dev), torch.from_numpy(z).to(dev), device=0).cpu().numpy()
    assert same(got, oracle_lib.glibc_batch(olib, "atan2", y, z))


def test_sin_odd_cos_even_bitwise():
    """k_prep's frame rotations take cos(-a) = cos(a) and sin(-a) = -sin(a) (two evaluations for
    four): both glibc and the restatement reduce |x| and apply the sign last, so the identities
    hold bit for bit (NaN aside) over headings, small, medium and large arguments."""
    olib = oracle_lib.load_oracle()
    x, _, _ = args(300_000, 3)
    x = x[np.isfinite(x)]
    for lib in ("restated", "glibc"):
        ev = (lambda k, a: ppamd.libm_eval(k, a)) if lib == "restated" else \
             (lambda k, a: oracle_lib.glibc_batch(olib, k, a))
        assert same(ev("cos", -x), ev("cos", x)), lib
        assert same(ev("sin", -x), -ev("sin", x)), lib

"""The HIP path's atan2 / sin / cos (csrc/farms_libm.h), host build.

They evaluate in double-double arithmetic and must round correctly: checked
against mpmath at 200 bits on random and special arguments.  The reference
calls glibc (vFlow.cpp:325, 366, 1007-1008, 1375-1377); glibc 2.35 misrounds a
small fraction of arguments, which is the only libm difference left between
the HIP path and the reference (counted here, and per stream in the GPU
parity tests).
"""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "aperture-robust-multiscale-optical-flow_amd", "build", "libfarms_libm_check.so")


@pytest.fixture(scope="module")
def lib():
    lib = ctypes.CDLL(LIB)
    lib.farms_libm_check.restype = ctypes.c_int64
    lib.farms_libm_check.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64] + [ctypes.c_void_p] * 2
    lib.farms_libm_fast_check.restype = ctypes.c_int64
    lib.farms_libm_fast_check.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int64, ctypes.c_void_p]
    return lib


def run(lib, fn, a, b=None):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(a if b is None else b, np.float64)
    cr, gl = np.empty_like(a), np.empty_like(a)
    diff = lib.farms_libm_check(fn, a.ctypes.data, b.ctypes.data, a.size, cr.ctypes.data, gl.ctypes.data)
    assert diff >= 0, "libm.so.6 not found"
    return diff, cr, gl


def samples(rng, n):
    ang = rng.uniform(-np.pi, np.pi, n)
    y = rng.standard_normal(n) * 10.0 ** rng.uniform(-5, 5, n)
    x = rng.standard_normal(n) * 10.0 ** rng.uniform(-5, 5, n)
    return ang, y, x


def test_correctly_rounded_vs_mpmath(lib):
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    rng = np.random.default_rng(2024)
    ang, y, x = samples(rng, 4000)
    # plus the neighbourhood of the reduction's boundaries and of k*pi/2
    edge = np.array([np.pi / 4 * k for k in range(-4, 5)] + [np.pi / 2 * k for k in range(-2, 3)], np.float64)
    edge = np.concatenate([np.nextafter(edge, np.inf), edge, np.nextafter(edge, -np.inf), [1e-9, -3e-12, 0.5]])
    ang = np.concatenate([ang, edge])
    _, s, _ = run(lib, 1, ang)
    _, c, _ = run(lib, 2, ang)
    _, a, _ = run(lib, 0, y, x)
    for i, v in enumerate(ang):
        m = mpmath.mpf(float(v))
        assert s[i] == float(mpmath.sin(m)), ("sin", v)
        assert c[i] == float(mpmath.cos(m)), ("cos", v)
    for i in range(y.size):
        assert a[i] == float(mpmath.atan2(mpmath.mpf(float(y[i])), mpmath.mpf(float(x[i])))), ("atan2", y[i], x[i])


def test_special_values_match_glibc(lib):
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-300, -1e-300, 1e300, 5e-324, 2.5, -3.0])
    Y, X = np.meshgrid(sp, sp)
    diff, _, _ = run(lib, 0, Y.ravel(), X.ravel())
    assert diff == 0  # IEEE special cases of atan2, signed zeros, infinities, NaN
    fin = sp[np.isfinite(sp) & (np.abs(sp) < 1e6)]
    for fn in (1, 2):
        diff, cr, gl = run(lib, fn, fin)
        assert diff == 0
        assert np.array_equal(np.signbit(cr), np.signbit(gl))


def test_glibc_misrounding_rate(lib):
    """Where the correctly rounded result and glibc differ, glibc is the one
    off (sampled against mpmath); the rate bounds the libm residual."""
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    rng = np.random.default_rng(7)
    ang, y, x = samples(rng, 300_000)
    rates = {}
    for fn, name, f in ((1, "sin", mpmath.sin), (2, "cos", mpmath.cos)):
        diff, cr, gl = run(lib, fn, ang)
        rates[name] = diff / ang.size
        for i in np.flatnonzero(cr != gl)[:40]:
            assert cr[i] == float(f(mpmath.mpf(float(ang[i]))))
    diff, cr, gl = run(lib, 0, y, x)
    rates["atan2"] = diff / y.size
    for i in np.flatnonzero(cr != gl)[:40]:
        assert cr[i] == float(mpmath.atan2(mpmath.mpf(float(y[i])), mpmath.mpf(float(x[i]))))
    print("glibc misrounding rates:", rates)
    assert all(r < 0.005 for r in rates.values()), rates


def test_fast_path_equals_full_evaluation(lib):
    """The Ziv fast paths (farms_libm.h: cheaper evaluation + rounding test,
    full double-double evaluation where the test cannot decide) return bitwise
    what the full evaluation alone returns, and fall back rarely (~2^-11)."""
    rng = np.random.default_rng(11)
    n = 1_000_000
    ang, y, x = samples(rng, n)
    k = rng.integers(-4, 5, n // 4)
    edge = k * (np.pi / 4) + rng.standard_normal(n // 4) * 10.0 ** rng.uniform(-16, -1, n // 4)
    fb = ctypes.c_int64(0)
    for fn, a, b in ((1, ang, ang), (2, ang, ang), (1, edge, edge), (2, edge, edge), (0, y, x),
                     (0, np.tan(ang), np.ones(n))):
        a = np.ascontiguousarray(a, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        diff = lib.farms_libm_fast_check(fn, a.ctypes.data, b.ctypes.data, a.size, ctypes.byref(fb))
        assert diff == 0, (fn, diff)
        assert fb.value / a.size < 1e-3, (fn, fb.value)

"""Exhaustive check of the floor form of the plain-BN element requant (plain-BN
build variant): the plain branches requantise every conv element and apply the ReLU right after
(layer2.c:139-210, layer4.c:113-130), so e = clamp(trunc(x / fac), 0, emax) equals
clamp(floor(x / fac), 0, emax), and the GPU computes it as
    bits(fmed3(fma(f32 bits (mbits + x), r, c), K, K + emax)) - bits(K),   K = 1.5 * 2^23
with constants the library chooses and verifies on the host (mibminet_test_floor_form).  This test
emulates those float operations bit-exactly for EVERY x in [-vmax, vmax] and compares with the C
semantics.  The fma is emulated in 80-bit long double: m * r + c needs at most 47 + log2|fac| bits,
exact for |fac| <= 2^17; larger factors are checked at every step boundary with exact fractions.
No GPU needed."""
import ctypes
from fractions import Fraction

import numpy as np
import pytest

from mibminet import lib

K = np.float32(12582912.0)
A = 128 * 128


def _floor_form(fac, emax, vmax):
    L = lib.load()
    fn = L.mibminet_test_floor_form
    fn.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    m, r, c = ctypes.c_int32(), ctypes.c_float(), ctypes.c_float()
    rc = fn(fac, emax, vmax, ctypes.addressof(m), ctypes.addressof(r), ctypes.addressof(c))
    return rc, m.value, np.float32(r.value), np.float32(c.value)


def _want(x, fac, emax):
    q = np.sign(x) * np.sign(fac) * (np.abs(x) // abs(fac))  # C's truncating division
    return np.clip(q, 0, emax)


def _check(fac, emax, vmax):
    rc, mbits, r, c = _floor_form(fac, emax, vmax)
    assert rc == 0, f"no floor form for fac={fac} emax={emax} vmax={vmax}"
    M = int(np.array([mbits], dtype=np.int32).view(np.float32)[0])
    assert (1 << 23) + vmax <= M <= (1 << 24) - 1 - vmax
    x = np.arange(-vmax, vmax + 1, dtype=np.int64)
    m = (M + x).astype(np.longdouble)  # exact: the f32 whose bits are mbits + x
    g = (m * np.longdouble(r) + np.longdouble(c)).astype(np.float32)  # == fmaf: exact, then one rounding
    e = np.clip(g, K, K + np.float32(emax)).astype(np.int64) - int(K)
    bad = np.nonzero(e != _want(x, fac, emax))[0]
    assert bad.size == 0, f"fac={fac}: x={x[bad[0]]} gives {e[bad[0]]}, C gives {_want(x[bad[0]:bad[0] + 1], fac, emax)}"


@pytest.mark.parametrize("fac", [1, -1, 2, 3, -7, 8, 50, -127, 1000, 8000, -65535, 131071])
def test_layer2_elements(fac):
    """Plain layer 2: elements clip to [0, 127]; |x| <= 64 * 128^2 + |offset >> 3|."""
    _check(fac, 127, 64 * A + 12345)


@pytest.mark.parametrize("fac", [1, -3, 16, 999, -4096, 100003])
def test_layer4_elements(fac):
    """Plain layer 4: elements clamp at 1024; |x| <= 16 * 128^2 + |offset >> 3|."""
    _check(fac, 1024, 16 * A + 777)


@pytest.mark.parametrize("fac", [1, -3, 16, 999, -4096])
def test_layer4_relu_only_elements(fac):
    """Plain layer 4 takes only the ReLU of the form, max(bits - bits(K), 0) (forward_wg.hpp,
    relu_sum8): exact up to the verified step 1024, and >= 1024 wherever the true element is (the
    window then saturates), for every reachable x."""
    emax, vmax = 1024, 16 * A + 777
    rc, mbits, r, c = _floor_form(fac, emax, vmax)
    assert rc == 0
    M = int(np.array([mbits], dtype=np.int32).view(np.float32)[0])
    x = np.arange(-vmax, vmax + 1, dtype=np.int64)
    g = ((M + x).astype(np.longdouble) * np.longdouble(r) + np.longdouble(c)).astype(np.float32)
    e = np.maximum(g.view(np.uint32).astype(np.int64) - int(np.array([K]).view(np.uint32)[0]), 0)
    q = np.sign(x) * np.sign(fac) * (np.abs(x) // abs(fac))
    want = np.maximum(q, 0)
    small = want <= emax
    assert np.array_equal(e[small], want[small]), fac
    assert (e[~small] >= emax).all(), fac


@pytest.mark.parametrize("fac", [(1 << 20) + 7, -(1 << 21) - 1, 2**31 - 1])
def test_large_factors_at_step_boundaries(fac):
    """|fac| > 2^17: exact fractions at both ends of every step interval (the form is monotone)."""
    emax, vmax = 127, 64 * A + 999
    rc, mbits, r, c = _floor_form(fac, emax, vmax)
    assert rc == 0
    M = int(np.array([mbits], dtype=np.int32).view(np.float32)[0])
    F = abs(fac)
    xs = {-vmax, vmax, -1, 0, 1}
    for k in range(-1, emax + 1):
        lo, hi = (k * F, k * F + F - 1) if fac > 0 else (-(k + 1) * F + 1, -k * F)
        xs.update(v for v in (lo, hi) if -vmax <= v <= vmax)
    for x in sorted(xs):
        exact = Fraction(M + x) * Fraction(float(r)) + Fraction(float(c))
        g = np.float32(float(exact))  # exact -> double (exact here) -> float: one rounding
        assert float(exact) == exact or abs(float(exact) - exact) < Fraction(1, 1 << 40)
        e = int(min(max(g, K), K + emax)) - int(K)
        assert e == int(_want(np.array([x]), fac, emax)[0]), (fac, x)

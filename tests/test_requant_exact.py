"""Exhaustive check of the exact requantisation: for a factor and an accumulator
bound vmax, the library picks a float reciprocal r (and for layers 1/3 the fma constant c); the
GPU then computes clip((int)RN(v * r)) or clip((int)fma(f32(1.5 * 2^23 + v), r, c)).  This test
emulates those float operations bit-exactly in NumPy for EVERY v in [-vmax, vmax] and compares
with C's clip(trunc(v / fac)).  No GPU: the reciprocal comes from the library's host code
(mibminet_test_reciprocal, include/mibminet_testing.h)."""
import ctypes

import numpy as np
import pytest

from mibminet import lib

CHUNK = 1 << 22


def _reciprocal(fac, vmax, magic):
    L = lib.load()
    fn = L.mibminet_test_reciprocal
    fn.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
    r, c = ctypes.c_float(), ctypes.c_float()
    rc = fn(fac, vmax, 128, int(magic), ctypes.addressof(r), ctypes.addressof(c))
    return rc, np.float32(r.value), np.float32(c.value)


def _check_exhaustive(fac, vmax, magic):
    rc, r, c = _reciprocal(fac, vmax, magic)
    assert rc == 0, f"no reciprocal for fac={fac} vmax={vmax}"
    for lo in range(-vmax, vmax + 1, CHUNK):
        v = np.arange(lo, min(lo + CHUNK, vmax + 1), dtype=np.int64)
        if magic:
            x = (np.float32(12582912.0) + v.astype(np.float32)).astype(np.float64)  # exact: |v| < 2^22
            q = (x * np.float64(r) + np.float64(c)).astype(np.float32)  # == fma: the sum is exact in f64
        else:
            q = v.astype(np.float32) * r  # float32 multiply, round to nearest even
        got = np.clip(q.astype(np.int64), -128, 127)  # truncating convert, then the saturating pack
        want = np.clip(np.sign(v) * np.sign(fac) * (np.abs(v) // abs(fac)), -128, 127)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"fac={fac} r={r!r}: v={v[bad[0]]} gives {got[bad[0]]}, C gives {want[bad[0]]}"


FACTORS = [1, -1, 3, 7, -13, 97, 255, 256, 4099, -8000, 65535, 65536, 65537, 100003,
           (1 << 20) + 7, -(1 << 20) - 9]


@pytest.mark.parametrize("fac", FACTORS)
def test_magic_form_layer1_range(fac):
    """Layers 1/3: fma form, |v| < 2^22 (layer 1's envelope)."""
    _check_exhaustive(fac, (1 << 22) - 1, True)


@pytest.mark.parametrize("fac", [5, -50, 1000, 8191, 65537, (1 << 20) + 7])
def test_mul_form_pooled_range(fac):
    """Layers 2/4/5: multiply form up to |v| < 2^24 (the pooled envelope)."""
    _check_exhaustive(fac, (1 << 24) - 1, False)


def test_small_vmax_uses_the_bound():
    """With a small reachable range even a huge factor has a reciprocal (everything maps to 0)."""
    rc, r, _ = _reciprocal(2**31 - 1, 16 * 128 * 128, False)
    assert rc == 0 and 0 < r < 1e-8


@pytest.mark.parametrize("fac", [2**31 - 1, -2**31, 2**24 + 1, -(2**23) - 3])
def test_int32_extremes(fac):
    _check_exhaustive(fac, (1 << 22) - 1, True)

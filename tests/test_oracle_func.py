"""Oracle pinning at the primitive level: the oracle's restatements of the reference's func/
kernels (src/cl/func/{dotp,xcorr,conv,transform,flip}.c), which its layers are built from, checked
against the expectations the reference's own func tests compute (test/cl/func/<name>/testcase.py),
at the sizes and constants those tests use.  The reference tests draw unseeded stimuli; here the
same distributions are drawn from fixed seeds.
"""
import ctypes

import numpy as np
import pytest

import oracle

vp, u, i32 = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int32


def _L():
    L = oracle.lib()
    L.or_func_dotp.argtypes = [vp, vp, u]
    L.or_func_dotp.restype = i32
    for n in ("or_func_xcorr", "or_func_conv"):
        getattr(L, n).argtypes = [vp, u, vp, u, vp]
        getattr(L, n).restype = None
    for n in ("or_func_xcorr_scale", "or_func_conv_scale"):
        getattr(L, n).argtypes = [vp, u, vp, u, i32, i32, vp]
        getattr(L, n).restype = None
    L.or_func_transform_32to8.argtypes = [vp, u, i32, u, vp]
    L.or_func_transform_32to8_bias.argtypes = [vp, u, i32, i32, u, vp]
    L.or_func_flip_2d_axis.argtypes = [vp, u, u, vp]
    return L


def _i8(rng, n):
    return rng.integers(-128, 128, size=n).astype(np.int8)


def _p(a):
    return a.ctypes.data


def _trunc_div(x, d):
    """C '/' (the testcases' float division then astype(int))."""
    q = np.abs(x) // abs(d)
    return np.where((x < 0) != (d < 0), -q, q)


@pytest.mark.parametrize("length", [22, 24, 1024, 1025, 1026, 1027, 1028, 1029, 1030, 1031])  # dotp/testcase.py:66
def test_dotp(length):
    rng = np.random.default_rng(length)
    a = rng.integers(-128, 127, size=length).astype(np.int8)  # np.random.randint(-128, 127) as the test
    b = rng.integers(-128, 127, size=length).astype(np.int8)
    assert _L().or_func_dotp(_p(a), _p(b), length) == int(np.dot(a.astype(np.int64), b.astype(np.int64)))


XCORR_SIZES = [(155, 16), (1021, 63), (1024, 63), (1188, 64), (4096, 128)]  # xcorr/testcase.py:59
SCALE_SIZES = [(155, 16), (1188, 64), (4096, 128)]  # {xcorr,conv}{_scale,}/testcase.py:59-62


@pytest.mark.parametrize("la,lb", XCORR_SIZES)
def test_xcorr(la, lb):
    rng = np.random.default_rng(la + lb)
    a, b = _i8(rng, la), _i8(rng, lb)
    want = np.correlate(a.astype(np.int64), b.astype(np.int64), mode="valid")
    r = np.zeros(la - lb + 1, np.int32)
    L = _L()
    L.or_func_xcorr(_p(a), la, _p(b), lb, _p(r))
    assert np.array_equal(r, want)
    r2 = np.zeros_like(r)  # xcorr.c:50-57: the shorter vector is always the kernel
    L.or_func_xcorr(_p(b), lb, _p(a), la, _p(r2))
    assert np.array_equal(r2, want)


@pytest.mark.parametrize("la,lb", SCALE_SIZES)
def test_conv(la, lb):
    rng = np.random.default_rng(la * lb)
    a, b = _i8(rng, la), _i8(rng, lb)
    want = np.convolve(a.astype(np.int64), b.astype(np.int64), mode="valid")
    r = np.zeros(la - lb + 1, np.int32)
    _L().or_func_conv(_p(a), la, _p(b), lb, _p(r))
    assert np.array_equal(r, want)


@pytest.mark.parametrize("kind", ["xcorr", "conv"])
@pytest.mark.parametrize("la,lb", SCALE_SIZES)
def test_scale(kind, la, lb):
    rng = np.random.default_rng(la + 7 * lb)
    a, b = _i8(rng, la), _i8(rng, lb)
    div = 128 * lb // 8  # {xcorr,conv}_scale/testcase.py:65-66
    off = 10 * div
    f = np.correlate if kind == "xcorr" else np.convolve
    raw = f(a.astype(np.int64), b.astype(np.int64), mode="valid")
    want = np.clip(_trunc_div(raw + off, div), -128, 127)
    r = np.zeros(la - lb + 1, np.int8)
    getattr(_L(), f"or_func_{kind}_scale")(_p(a), la, _p(b), lb, div, off, _p(r))
    assert np.array_equal(r, want)


@pytest.mark.parametrize("size", [1024, 1025, 1026, 1027])  # transform/testcase.py:69
def test_transform(size):
    rng = np.random.default_rng(size)
    x = rng.integers(-2560, 2561, size=size).astype(np.int32)  # max_val=2560, SCALE_FACTOR 10, BIAS 50
    pad = (size + 3) // 4 * 4
    L = _L()
    r = np.full(pad, 0x55, np.int8)
    L.or_func_transform_32to8(_p(x), size, 10, 1, _p(r))
    assert np.array_equal(r[:size], np.clip(_trunc_div(x.astype(np.int64), 10), -128, 127))
    assert not r[size:].any()  # the partial last pack is zero-filled
    rb = np.full(pad, 0x55, np.int8)
    L.or_func_transform_32to8_bias(_p(x), size, 10, 50, 1, _p(rb))
    assert np.array_equal(rb[:size], np.clip(_trunc_div(x.astype(np.int64) + 50, 10), -128, 127))
    assert not rb[size:].any()
    # stride: every third element (layer code passes 1; the primitive supports any)
    xs = np.repeat(x, 3)
    r3 = np.zeros(pad, np.int8)
    L.or_func_transform_32to8(_p(xs), size, 10, 3, _p(r3))
    assert np.array_equal(r3, r)


@pytest.mark.parametrize("outer", [16, 17, 18, 19])
@pytest.mark.parametrize("inner", [256, 257, 258, 259])  # flip/testcase.py:72-73
def test_flip(outer, inner):
    rng = np.random.default_rng(outer * 1000 + inner)
    x = rng.integers(-128, 127, size=(outer, inner)).astype(np.int8)
    ia, oa = (inner + 3) // 4 * 4, (outer + 3) // 4 * 4
    xin = np.zeros((outer, ia), np.int8)  # header_file.align_array(inp): zero fill
    xin[:, :inner] = x
    want = np.zeros((inner, oa), np.int8)  # align_array(transpose(inp))
    want[:, :outer] = x.T
    r = np.full((inner, oa), 0x55, np.int8)
    _L().or_func_flip_2d_axis(_p(xin), outer, inner, _p(r))
    assert np.array_equal(r, want)


@pytest.mark.parametrize("length", [22, 23, 1024, 1025])  # dotp_slow/testcase.py:66-67
@pytest.mark.parametrize("a_stride,b_stride", [(1, 1), (4, 1), (8, 4)])
def test_dotp_slow(length, a_stride, b_stride):
    """func_dotp_slow (dotp.c:172): the test's [length][stride] arrays, expectation
    np.dot(vec_a[:, 0], vec_b[:, 0])."""
    L = _L()
    L.or_func_dotp_slow.argtypes = [vp, u, vp, u, u]
    L.or_func_dotp_slow.restype = i32
    rng = np.random.default_rng(length * 100 + a_stride * 10 + b_stride)
    a = rng.integers(-128, 127, size=(length, a_stride)).astype(np.int8)
    b = rng.integers(-128, 127, size=(length, b_stride)).astype(np.int8)
    want = int(np.dot(a[:, 0].astype(np.int64), b[:, 0].astype(np.int64)))
    assert L.or_func_dotp_slow(_p(a), a_stride, _p(b), b_stride, length) == want


@pytest.mark.parametrize("C,T,stress,reorder", [(22, 1125, False, True), (22, 1125, True, True),
                                                (64, 1000, True, True), (22, 1125, True, False)])
def test_layer4_flip_and_noflip_branches_agree(C, T, stress, reorder):
    """Layer 4 restated twice, from the reference's two build branches: FLIP_LAYERS (layer4.c:51-149,
    dotp over rows of the flipped [T8][F2] input: or_layer4) and without it (layer4.c:380-505,
    func_dotp_slow down the columns of the unflipped [F2][T8_ALIGN] input: or_layer4_noflip).  They
    must agree on every output, including both clip rails and negative truncation (stress params)."""
    from mibminet.params import ParamSet

    ps = ParamSet.synthetic(seed=C + T + stress, C=C, T=T, stress=stress, reorder_bn=reorder)
    co = oracle.COracle(ps)
    L = co.L
    L.or_layer4_noflip.argtypes = [vp, vp, vp]
    L.or_layer4_noflip.restype = None
    d = ps.dims
    rng = np.random.default_rng(C * T)
    for trial in range(6):
        lo, hi = [(-128, 128), (-60, 60), (-128, -100), (100, 128), (-8, 8), (-128, 128)][trial]
        y3 = np.zeros((d.F2, d.T8_ALIGN), np.int8)
        y3[:, : d.T8] = rng.integers(lo, hi, size=(d.F2, d.T8))
        flipped = co.layer3_flip(y3)
        a = co.layer4(flipped)
        b = np.empty((d.F2, d.T64_ALIGN), np.int8)
        L.or_layer4_noflip(co.pref, y3.ctypes.data, b.ctypes.data)
        np.testing.assert_array_equal(a[:, : d.T64], b[:, : d.T64])

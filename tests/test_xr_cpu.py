"""Exact-division mode selection on the host (no GPU): which parameter sets run the float requant
kernels, which the exact-division kernels (Cfg::XR), and which the loader refuses because the
reference's own int32 arithmetic is undefined on them (overflow, zero divisor, INT_MIN / -1).

The boundaries are recomputed here from the reference's evaluation order (layer1.c:90-91,
layer2.c:97-111, layer4.c:99-138) with Python integers, independently of the loader's C++.
"""
import struct

import numpy as np
import pytest

from mibminet import lib
from mibminet.params import HEADER_SIZE, ParamSet, appendix_b_net, dot_ranges, tdiv

I32_MIN, I32_MAX = -(2 ** 31), 2 ** 31 - 1


def _load(ps):
    L = lib.load()
    b = ps.to_blob()
    rc = L.net_params_load(b, len(b))
    if rc == 0:
        lib._loaded = ps
        return rc, lib.params_exact_division()
    return rc, None


@pytest.fixture(autouse=True)
def _unload():
    yield
    lib.params_unload()


def test_xdiv_host_matches_c_division():
    """The exact-division sequence (emulated on the host) against C division: every divisor class
    (+-1, powers of two and their neighbours, int32 extremes, random), dividends around every
    quotient step of the clipped range and at the int32 ends."""
    rng = np.random.default_rng(2)
    ds = [1, -1, 2, -2, 3, 7, 128, -129, 1 << 16, (1 << 16) + 1, (1 << 24) - 1, 1 << 24, 1 << 30, I32_MAX,
          -I32_MAX, I32_MIN] + [int(v) for v in rng.integers(I32_MIN, I32_MAX, 300) if v]
    for d in ds:
        ks = np.arange(-131, 132, dtype=np.int64)
        e = np.concatenate([(ks[:, None] * d + np.arange(-2, 3)[None, :]).ravel(),
                            rng.integers(I32_MIN, I32_MAX + 1, 4000), [I32_MIN, I32_MIN + 1, -1, 0, 1, I32_MAX]])
        e = e[(e >= I32_MIN) & (e <= I32_MAX)]
        if d == -1:
            e = e[e != I32_MIN]
        got = lib.xdiv_host(e.astype(np.int32), d).astype(np.int64)
        want = np.array([tdiv(int(v), d) for v in e], np.int64)
        assert np.array_equal(got, want), d


def test_calibrated_sets_stay_on_the_float_kernels():
    """The benchmark and parity sets keep today's float requant kernels."""
    for seed in range(12):
        for kw in (dict(), dict(stress=True), dict(C=64, T=1000), dict(weight_bits=4), dict(reorder_bn=False),
                   dict(clip_balanced=True), dict(C=64, T=480, reorder_bn=False)):
            rc, xr = _load(ParamSet.synthetic(seed=seed, **kw))
            assert rc == 0 and xr is False, (seed, kw)
    net, cfg, _ = appendix_b_net(0)
    assert _load(ParamSet.from_quantlab(net, cfg)) == (0, False)


def test_extreme_sets_load_exact():
    for rb in (True, False):
        for C, T in ((22, 1125), (64, 1000), (64, 480)):
            assert _load(ParamSet.synthetic_extreme(5, C=C, T=T, reorder_bn=rb)) == (0, True), (rb, C, T)


@pytest.mark.parametrize("f", [0, 5, 13])
def test_layer1_boundaries(f):
    """Layer 1 (acc + off, layer1.c:90-91): the float envelope ends where |dot + off| reaches 2^22
    (then the exact kernels), and the loader refuses exactly where the int32 sum can overflow."""
    ps0 = ParamSet.synthetic(seed=2)
    lo, hi = dot_ranges(ps0)[0][f]

    def at(off, fac=None):
        ps = ParamSet.synthetic(seed=2)
        ps.l1_offset[f] = off
        if fac is not None:
            ps.l1_factor[f] = fac
        return _load(ps)

    # factor 2^15: the outputs still vary near |v| = 2^22 (a rail would be folded, below)
    F = 1 << 15
    assert at((1 << 22) - 1 - hi, F) == (0, False)
    assert at((1 << 22) - hi, F) == (0, True)
    assert at(-(1 << 22) + 1 - lo, F) == (0, False)
    assert at(-(1 << 22) - lo, F) == (0, True)
    # at the int32 ends a factor with the output step 99 -> 100 inside the reachable range
    Fe = (I32_MAX - (hi - lo) // 2) // 100
    assert at(I32_MAX - hi, Fe) == (0, True)
    assert at(I32_MAX - hi + 1)[0] == lib.NET_ERR_RANGE
    assert at(I32_MIN - lo, -Fe) == (0, True)
    assert at(I32_MIN - lo - 1)[0] == lib.NET_ERR_RANGE
    # INT_MIN reachable: / -1 is undefined in C, / -2 is not (every output then sits on the +127
    # rail: folded, float kernels)
    assert at(I32_MIN - lo, -1)[0] == lib.NET_ERR_RANGE
    assert at(I32_MIN - lo, -2) == (0, False) and lib.folded_filters() == 1
    # the calibrated factor with the offset at the int32 end: a rail, folded
    assert at(I32_MAX - hi) == (0, False) and lib.folded_filters() == 1


@pytest.mark.parametrize("name,f", [("l2", 3), ("l4", 9)])
def test_pooled_boundaries(name, f):
    """REORDER_BN layers 2 and 4 (sum_8 max(v, -(off >> 3)) + off, layer2.c:97-111): float while
    the pooled sum stays below 2^24, exact beyond, refused where a partial sum or sum + off leaves
    int32 (off = -2^31: eight thresholds of 2^28)."""
    ps0 = ParamSet.synthetic(seed=4)
    lo, hi = dot_ranges(ps0)[1 if name == "l2" else 2][f]

    def at(off, fac=None):
        ps = ParamSet.synthetic(seed=4)
        getattr(ps, f"{name}_offset")[f] = off
        if fac is not None:
            getattr(ps, f"{name}_factor")[f] = fac
        return _load(ps)

    # factors that keep the outputs varying (a rail would be folded onto the float kernels)
    assert at((1 << 24) - 1 - 8 * hi, 1 << 17) == (0, False)
    assert at((1 << 24) - 8 * hi, 1 << 17) == (0, True)
    assert at(I32_MAX - 8 * hi, (I32_MAX - 4 * (hi - lo)) // 100) == (0, True)
    assert at(I32_MAX - 8 * hi) == (0, False) and lib.folded_filters() == 1
    assert at(I32_MAX - 8 * hi + 1)[0] == lib.NET_ERR_RANGE
    # every element suppressed: sum = 8 thr + off = off & 7, on the float kernels
    assert at(I32_MIN + 8) == (0, False)
    assert at(I32_MIN + 15) == (0, False)
    assert at(I32_MIN)[0] == lib.NET_ERR_RANGE  # 8 * 2^28 overflows


def test_plain_layer4_sum_overflow():
    """Plain layer 4 sums eight unclipped elements (layer4.c:113-130): refused when 8 elements can
    pass INT32_MAX."""
    ps0 = ParamSet.synthetic(seed=6, reorder_bn=False)
    lo, hi = dot_ranges(ps0)[2][2]

    def at(off3):
        ps = ParamSet.synthetic(seed=6, reorder_bn=False)
        ps.l4_factor[2] = 8  # factor >> 3 == 1: element = v + (off >> 3)
        ps.l4_offset[2] = 8 * off3
        return _load(ps)

    limit = I32_MAX // 8 - hi  # largest off3 with 8 (hi + off3) <= INT32_MAX
    assert at(limit) == (0, False) and lib.folded_filters() == 1  # every element >= 127: a rail
    assert at(limit + 1)[0] == lib.NET_ERR_RANGE


def test_zero_factors_refused():
    """A zero divisor (C division by zero) is refused; ParamSet refuses to build one, so the blob is
    patched."""
    L = lib.load()
    ps = ParamSet.synthetic(seed=1)
    blob = bytearray(ps.to_blob())
    struct.pack_into("<i", blob, HEADER_SIZE + 4 * 3, 0)  # net_l1_factor[3]
    assert L.net_params_load(bytes(blob), len(blob)) == lib.NET_ERR_RANGE
    ps = ParamSet.synthetic(seed=1, reorder_bn=False)
    ps.l2_factor[0] = 8
    blob = bytearray(ps.to_blob())
    C_ALIGN = ps.dims.C_ALIGN
    off = HEADER_SIZE + 2 * 64 + 16 * C_ALIGN  # net_l2_factor[0]
    struct.pack_into("<i", blob, off, 7)  # 7 >> 3 == 0: the plain branch divides by zero
    assert L.net_params_load(bytes(blob), len(blob)) == lib.NET_ERR_RANGE


def test_pool_constants_keep_the_pooled_sum():
    """The biased ReLU pooling (forward_common.hpp, pool8b) with the loader's clamped threshold and
    offset term equals the reference's sum_8 max(v, -(off >> 3)) + off (layer2.c:97-111,
    layer4.c:99-130) for offsets across the whole int32 range, including thresholds past either
    end of the conv range (the kernels' biased values must not wrap, so the threshold is clamped)."""
    import ctypes
    L = lib.load()
    rng = np.random.default_rng(8)
    for layer, V in ((2, 1 << 20), (4, 1 << 18)):
        vlo = -((V // (128 * 128)) * 128 * 127)  # 64 (16) taps of (-128) x 127
        offs = [I32_MIN + 8, I32_MIN + 15, -(1 << 30), -8 * V - 64, -8 * V, -8 * V + 8, -1, 0, 7, 8, 8 * V,
                8 * V + 9, 1 << 30, I32_MAX - 8 * V] + [int(o) for o in rng.integers(I32_MIN + 8, I32_MAX - 8 * V, 200)]
        thr_c, offm = ctypes.c_int32(), ctypes.c_int32()
        for off in offs:
            assert L.mibminet_test_pool_consts(off, layer, ctypes.byref(thr_c), ctypes.byref(offm)) == 0
            assert -V <= thr_c.value <= V
            thr = -(off >> 3)
            for _ in range(20):
                v = rng.integers(vlo, V + 1, 8)
                v[: rng.integers(0, 3)] = rng.choice([vlo, V, 0, thr_c.value])
                want = int(np.maximum(v, thr).sum()) + off
                if not I32_MIN <= want <= I32_MAX:
                    continue
                got = (int(np.maximum(v - thr_c.value, 0).sum()) + offm.value) % (1 << 32)
                assert (got - (1 << 32) if got > I32_MAX else got) == want, (layer, off, v.tolist())


def _fold(ps):
    """Python restatement of the loader's constant-filter folding (mibminet.hip,
    fold_constant_filters): a filter whose clipped output is one value y over its whole reachable
    numerator range gets zero weights and offset/factor that reproduce y."""
    import copy

    q = copy.deepcopy(ps)
    lo_clip = -127 if ps.clip_balanced else -128
    r1, r2, r4 = dot_ranges(ps)
    F2, CA = ps.dims.F2, ps.dims.C_ALIGN
    w1 = q.l1_weight_align.reshape(F2, CA)

    def out(v, fac):
        return min(127, max(lo_clip, tdiv(v, fac)))

    n = 0
    for f in range(F2):
        off, fac = int(ps.l1_offset[f]), int(ps.l1_factor[f])
        lo, hi = r1[f]
        if out(lo + off, fac) == out(hi + off, fac):
            w1[f] = 0
            q.l1_offset[f], q.l1_factor[f] = out(lo + off, fac), 1
            n += 1
        for name, rr, w in (("l2", r2, q.l2_weight_reverse), ("l4", r4, q.l4_weight)):
            off, fac = int(getattr(ps, f"{name}_offset")[f]), int(getattr(ps, f"{name}_factor")[f])
            lo, hi = rr[f]
            if ps.reorder_bn:
                thr = -(off >> 3)
                a, b = out(8 * max(lo, thr) + off, fac), out(8 * max(hi, thr) + off, fac)
                if a != b:
                    continue
                y, o2, f2 = a, abs(a), (-1 if a < 0 else 1)
            else:
                e = sorted((tdiv(lo + (off >> 3), fac >> 3), tdiv(hi + (off >> 3), fac >> 3)))
                if e[1] > 0 and e[0] < 127 and e[0] != e[1]:
                    continue
                y = min(127, max(0, e[0]))
                o2, f2 = 8 * y, 8
            w[f] = 0
            getattr(q, f"{name}_offset")[f], getattr(q, f"{name}_factor")[f] = o2, f2
            n += 1
    return q, n


@pytest.mark.parametrize("rb", [True, False])
@pytest.mark.parametrize("cb", [False, True])
def test_constant_filters_fold_onto_the_float_kernels(rb, cb):
    """Item 6 of round 5's verdict: per-filter classification.  A set whose out-of-envelope filters
    all sit on a rail (or at zero, or suppressed by the REORDER_BN threshold) loads on the float
    kernels, the compiled shapes and the general kernels alike; one varying filter past the
    envelope still takes it to exact division, and params_info names that filter."""
    for C, T in ((22, 1125), (64, 480), (19, 480)):
        ps = ParamSet.synthetic_extreme(3 + C, C=C, T=T, reorder_bn=rb, clip_balanced=cb, mids=0)
        assert _load(ps) == (0, False), (C, T)
        _, n = _fold(ps)
        assert lib.folded_filters() == n >= 15
        ps1 = ParamSet.synthetic_extreme(3 + C, C=C, T=T, reorder_bn=rb, clip_balanced=cb, mids=1)
        assert _load(ps1) == (0, True), (C, T)
        info = lib.params_info()
        if info["path"] == "exact":
            folded, _ = _fold(ps1)
            layer, f = info["layer"], info["filter"]
            # the named filter is not one the loader folded: its parameters are unchanged
            name = f"l{layer}"
            assert getattr(folded, f"{name}_factor")[f] == getattr(ps1, f"{name}_factor")[f]
            assert getattr(folded, f"{name}_offset")[f] == getattr(ps1, f"{name}_offset")[f]


@pytest.mark.parametrize("rb", [True, False])
def test_folding_keeps_the_oracle_outputs(rb):
    """The folded set computes the original's outputs (C oracle, every layer), on random trials and
    on the all-rail inputs; the loader folds the same filters."""
    import oracle

    ps = ParamSet.synthetic_extreme(29, C=22, T=1125, reorder_bn=rb, mids=6)
    folded, n = _fold(ps)
    assert n >= 14
    assert _load(ps)[0] == 0 and lib.folded_filters() == n
    rng = np.random.default_rng(4)
    x = rng.integers(-128, 128, size=(24, 22, 1125)).astype(np.int8)
    x[0], x[1], x[2] = 127, -128, 0
    from mibminet.params import pack_trials
    xp = pack_trials(x)
    a, b = oracle.COracle(ps), oracle.COracle(folded)
    assert np.array_equal(a.batch(xp, nthreads=4), b.batch(xp, nthreads=4))
    d = ps.dims
    for t in range(3):
        xa = oracle.to_tc_align(x[t], d.C_ALIGN)
        y1 = a.layer1(xa)
        assert np.array_equal(y1, b.layer1(xa))
        y2 = a.layer2(y1)
        assert np.array_equal(y2, b.layer2(y1))
        y3t = a.layer3_flip(a.layer3(y2))
        assert np.array_equal(a.layer4(y3t), b.layer4(y3t))

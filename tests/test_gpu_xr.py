"""Exact-division kernels (Cfg::XR): parameter sets outside the float requant envelope.

The reference computes every requant as C's int32 ``(acc + off) / fac`` (layer1.c:90-91,
layer2.c:110-111, layer4.c:129-130, transform.c:47), for any int32 offsets and factors.  Sets whose
offsets or factors leave the float envelope run kernels that divide exactly in
integers (forward_common.hpp, xdiv).  These tests check:

* the device division itself against C division over the whole int32 range for a few divisors and
  around every clip boundary for many more;
* whole networks with extreme parameters (ParamSet.synthetic_extreme: offsets near +-2^30, factors
  1 and +-(2^31 - 1), threshold-suppressed filters, |offsets| past 2^22) against the C oracle, for
  every shape, both BN branches, both clip modes, int8 and int4 weights, time-major and
  channel-major input, the float-input entry (against the two-pass chain) and the reference's
  single-trial and per-layer entry points.
The committed fixture ``fixture_xr22.npz`` runs through test_gpu_parity.py's fixture tests too.
"""
import os

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu
I32_MIN, I32_MAX = -(2 ** 31), 2 ** 31 - 1
NT = min(16, os.cpu_count() or 1)


@pytest.mark.parametrize("d", [1, -3, I32_MAX])
def test_xdiv_gpu_every_int32(d, gpu):
    """The device xdiv equals C division for all 2^32 dividends (INT_MIN / -1: RISC-V's INT_MIN,
    which the loader refuses anyway)."""
    assert lib.xdiv_gpu_mismatches(d, I32_MIN, 2 ** 32) == 0


def test_xdiv_gpu_boundaries(gpu):
    """Many divisors, each over the dividends around every quotient step of the clipped range
    (k d - 2 .. k d + 2 for |k| <= 130) and the int32 ends."""
    rng = np.random.default_rng(5)
    ds = [2, -2, 7, 127, -128, 255, 1 << 16, (1 << 16) + 1, (1 << 20) + 7, 1 << 24, (1 << 24) + 1, 1 << 30,
          -(1 << 31) + 1, I32_MIN] + [int(v) for v in rng.integers(I32_MIN, I32_MAX, 24) if v != 0]
    for d in ds:
        for k in range(-130, 131):
            lo = max(I32_MIN, k * d - 2)
            hi = min(I32_MAX, k * d + 2)
            if lo <= hi:
                assert lib.xdiv_gpu_mismatches(d, lo, hi - lo + 1) == 0, (d, k)
        assert lib.xdiv_gpu_mismatches(d, I32_MIN, 1 << 20) == 0, d
        assert lib.xdiv_gpu_mismatches(d, I32_MAX - (1 << 20) + 1, 1 << 20) == 0, d


def _cases():
    out = []
    for i, (C, T) in enumerate(((22, 1125), (64, 1000), (64, 480))):
        for rb in (True, False):
            for cb in (False, True):
                out.append(dict(seed=40 + 4 * i + 2 * rb + cb, C=C, T=T, rb=rb, cb=cb, w=4 if (i + cb) % 3 == 2 else 8))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "{C}x{T}-rb{rb:d}-cb{cb:d}-w{w}".format(**c))
def test_extreme_nets_vs_oracle(case, gpu):
    """Time-major and channel-major batches of an extreme set, both against the C oracle."""
    import torch

    ps = ParamSet.synthetic_extreme(case["seed"], C=case["C"], T=case["T"], weight_bits=case["w"],
                                    reorder_bn=case["rb"], clip_balanced=case["cb"])
    lib.params_load(ps)
    assert lib.params_exact_division()
    rng = np.random.default_rng(case["seed"])
    B = 97
    x = rng.integers(-128, 128, size=(B, case["C"], case["T"])).astype(np.int8)
    x[: B // 3] = rng.integers(-60, 60, size=(B // 3, case["C"], case["T"]))
    x[-1] = 127
    x[-2] = -128
    xp = pack_trials(x)
    want = oracle.COracle(ps).batch(xp, nthreads=NT)
    got = lib.forward_torch(torch.from_numpy(xp).cuda()).cpu().numpy()
    assert np.array_equal(got, want)
    got_ct = lib.forward_ct_torch(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(got_ct, want)


@pytest.mark.parametrize("rb", [True, False])
def test_extreme_single_trial_and_layers(rb, gpu):
    """The reference's own entry points (net_model_compute, net_layer1..5) on an extreme set."""
    ps = ParamSet.synthetic_extreme(77 + rb, C=22, T=1125, reorder_bn=rb)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    rng = np.random.default_rng(3)
    d = ps.dims
    for _ in range(3):
        xa = oracle.to_tc_align(rng.integers(-128, 128, size=(d.C, d.T)).astype(np.int8), d.C_ALIGN)
        y1 = co.layer1(xa)
        np.testing.assert_array_equal(lib.net_layer1(xa), y1)
        y2 = co.layer2(y1)
        np.testing.assert_array_equal(lib.net_layer2(y1), y2)
        y3 = co.layer3(y2)
        np.testing.assert_array_equal(lib.net_layer3(y2), y3)
        y3t = co.layer3_flip(y3)
        y4 = co.layer4(y3t)
        np.testing.assert_array_equal(lib.net_layer4(y3t), y4)
        np.testing.assert_array_equal(lib.net_layer5(y4), co.layer5(y4))
        np.testing.assert_array_equal(lib.net_model_compute(xa), co.model(xa))
    # arbitrary int8 layer inputs (the per-layer API takes any int8), both rails included
    y1 = rng.integers(-128, 128, size=(d.F1, d.T_ALIGN)).astype(np.int8)
    y1[:, d.T:] = 0
    np.testing.assert_array_equal(lib.net_layer2(y1), co.layer2(y1))
    y3t = rng.integers(-128, 128, size=(d.T8 * d.F2,)).astype(np.int8)
    buf = np.zeros(d.F2 * d.T8_ALIGN, np.int8)
    buf[: d.T8 * d.F2] = y3t
    np.testing.assert_array_equal(lib.net_layer4(buf), co.layer4(buf))


@pytest.mark.parametrize("C,T,rb", [(22, 1125, True), (64, 1000, True), (22, 1125, False)])
def test_extreme_f32_matches_chain(C, T, rb, gpu):
    """Float input into the exact-division kernel equals the two-pass chain (quantiser, then the
    time-major forward) and the oracle on the quantised trials."""
    import torch

    ps = ParamSet.synthetic_extreme(91, C=C, T=T, reorder_bn=rb)
    lib.params_load(ps)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.normal(0.0, 1.2, size=(64, C, T)).astype(np.float32)).cuda()
    y = lib.forward_f32_torch(x, 2.0).cpu().numpy()
    xq = lib.quantize_input_torch(x, 2.0)
    assert np.array_equal(y, lib.forward_torch(xq).cpu().numpy())
    assert np.array_equal(y, oracle.COracle(ps).batch(xq.cpu().numpy(), nthreads=NT))


def test_extreme_full_batch(gpu):
    """Config B's full batch (65,536 trials) on an extreme set: sampled trials against the oracle,
    channel-major equal to time-major on every trial, and determinism."""
    import torch

    ps = ParamSet.synthetic_extreme(123, C=22, T=1125)
    lib.params_load(ps)
    rng = np.random.default_rng(9)
    B = 65536
    x = torch.randint(-128, 128, (B, 22, 1125), dtype=torch.int8, device="cuda")
    xp = torch.zeros((B, lib.trial_stride()), dtype=torch.int8, device="cuda")
    xp[:, : 22 * 1125] = x.transpose(1, 2).reshape(B, -1)
    y = lib.forward_torch(xp)
    y2 = lib.forward_torch(xp)
    yc = lib.forward_ct_torch(x)
    assert torch.equal(y, y2) and torch.equal(y, yc)
    idx = np.concatenate([np.arange(16), B - 16 + np.arange(16), rng.choice(B, 256, replace=False)])
    xs = xp[torch.from_numpy(idx).cuda()].cpu().numpy()
    assert np.array_equal(y.cpu().numpy()[idx], oracle.COracle(ps).batch(xs, nthreads=NT))


@pytest.mark.parametrize("C,T,rb,cb", [(22, 1125, True, False), (22, 1125, False, True), (64, 1000, True, True),
                                       (64, 480, False, False), (19, 480, True, False), (38, 1125, False, False)])
def test_folded_rail_sets_on_the_float_kernels(C, T, rb, cb, gpu):
    """Sets whose out-of-envelope filters are all constant load on the float kernels with those
    filters folded (mibminet.hip, fold_constant_filters); the outputs equal the C oracle on the set
    as given, batched (both layouts) and through the reference's single-trial and layer entries."""
    import torch

    ps = ParamSet.synthetic_extreme(61 + C, C=C, T=T, reorder_bn=rb, clip_balanced=cb, mids=0)
    lib.params_load(ps)
    assert not lib.params_exact_division() and lib.folded_filters() >= 15
    rng = np.random.default_rng(C + T)
    B = 67
    x = rng.integers(-128, 128, size=(B, C, T)).astype(np.int8)
    x[-1] = 127
    x[-2] = -128
    xp = pack_trials(x)
    co = oracle.COracle(ps)
    want = co.batch(xp, nthreads=NT)
    assert np.array_equal(lib.forward_torch(torch.from_numpy(xp).cuda()).cpu().numpy(), want)
    assert np.array_equal(lib.forward_ct_torch(torch.from_numpy(x).cuda()).cpu().numpy(), want)
    d = ps.dims
    xa = oracle.to_tc_align(x[0], d.C_ALIGN)
    y1 = co.layer1(xa)
    np.testing.assert_array_equal(lib.net_layer1(xa), y1)
    y2 = co.layer2(y1)
    np.testing.assert_array_equal(lib.net_layer2(y1), y2)
    y3t = co.layer3_flip(co.layer3(y2))
    y4 = co.layer4(y3t)
    np.testing.assert_array_equal(lib.net_layer4(y3t), y4)
    np.testing.assert_array_equal(lib.net_model_compute(xa), co.model(xa))


def test_xr_divisor_extremes_on_varying_filters(gpu):
    """The exact-division kernels' divisor magics at their ends: layer-1 filters with
    factors 1, -1, 2^31 - 1 and -(2^31 - 1) whose outputs vary (so none is folded), in a set that
    runs exact division, against the oracle.  Crafted trials reach each filter's range end
    (dot = its maximum or minimum), where trunc(v / +-(2^31 - 1)) = +-1."""
    import torch

    I32_MAX, I32_MIN = 2 ** 31 - 1, -(2 ** 31)
    ps = ParamSet.synthetic_extreme(314, C=22, T=1125, mids=6)
    from mibminet.params import dot_ranges
    r1 = dot_ranges(ps)[0]
    w1 = ps.w1().astype(np.int64)  # [F][C]
    picks = {}
    for f, (fac, off_of) in zip((1, 4, 7, 10), (
            (1, lambda lo, hi: -((lo + hi) // 2)),
            (-1, lambda lo, hi: -((lo + hi) // 2)),
            (I32_MAX, lambda lo, hi: I32_MAX - hi),
            (-I32_MAX, lambda lo, hi: I32_MIN + 1 - lo))):
        lo, hi = r1[f]
        ps.l1_factor[f] = np.int32(fac)
        ps.l1_offset[f] = np.int32(off_of(lo, hi))
        picks[f] = fac
    ps.__post_init__()
    lib.params_load(ps)
    assert lib.params_exact_division()
    rng = np.random.default_rng(5)
    B = 40
    x = rng.integers(-128, 128, size=(B, 22, 1125)).astype(np.int8)
    for i, f in enumerate((7, 10)):  # every sample at the filter's dot maximum (7) / minimum (10)
        top = np.where(w1[f] > 0, 127, -128) if f == 7 else np.where(w1[f] > 0, -128, 127)
        x[i] = top[:, None].astype(np.int8)
    xp = pack_trials(x)
    co = oracle.COracle(ps)
    assert np.array_equal(lib.forward_torch(torch.from_numpy(xp).cuda()).cpu().numpy(), co.batch(xp, nthreads=NT))
    d = ps.dims
    for i in (0, 1, 2):
        xa = oracle.to_tc_align(x[i], d.C_ALIGN)
        y1 = lib.net_layer1(xa)
        np.testing.assert_array_equal(y1, co.layer1(xa))
        if i == 0:
            assert (y1[7, : d.T] == 1).all()   # trunc(INT32_MAX / INT32_MAX)
        if i == 1:
            assert (y1[10, : d.T] == 1).all()  # trunc((INT32_MIN + 1) / -INT32_MAX)

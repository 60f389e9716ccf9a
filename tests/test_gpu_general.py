"""The general-geometry kernels (forward_gen.hpp): every network QuantLab's loaders produce.

MI-BMInet's channel selection cuts the input to C = len(cs) channels
(QuantLab/quantlab/PhysionetMMMI/edgeEEGNet/preprocess.py:86-87) and the PhysioNet loader trains
2- and 3-class networks (get_data.py:73-82) on 480- or 960-sample windows (get_data.py:156-159);
gen_net_header.py:78-89 emits NET_C, NET_T and NET_N for any of them.  Each is checked against
the C oracle (oracle/oracle.c, the reference's layer1..5 restated) through the batched
time-major and channel-major entries, the float-input entry, the single-trial net_model_compute
and every per-layer entry point.  The compiled geometries are also forced onto the general
kernels (mibminet_test_force_general) so that both kernel families meet the same oracle on the
same sets.
"""
import os

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu
NTH = min(16, os.cpu_count() or 1)


def _ct(torch, x_ct, offset=0):
    """[B][C][T] int8 on the device, starting `offset` bytes into its allocation."""
    B, C, T = x_ct.shape
    flat = torch.zeros(offset + B * C * T + 64, dtype=torch.int8, device="cuda")
    flat[offset: offset + B * C * T] = torch.from_numpy(np.ascontiguousarray(x_ct, np.int8).ravel()).cuda()
    return flat[offset: offset + B * C * T].view(B, C, T)


def _check_all_entries(ps, B, seed, offset=1, layers=True):
    import torch

    lib.params_load(ps)
    assert lib.params_info()["path"] == "general"
    d = ps.dims
    co = oracle.COracle(ps)
    rng = np.random.default_rng(seed)
    x_ct = rng.integers(-128, 128, size=(B, d.C, d.T)).astype(np.int8)
    xp = pack_trials(x_ct)
    want = co.batch(xp, nthreads=NTH)
    got = lib.forward_torch(torch.from_numpy(xp).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, want, err_msg="time-major")
    got_ct = lib.forward_ct_torch(_ct(torch, x_ct, offset)).cpu().numpy()
    np.testing.assert_array_equal(got_ct, want, err_msg="channel-major")
    # the reference's single-trial entry and its per-layer entries
    x0 = oracle.to_tc_align(x_ct[0], d.C_ALIGN)
    np.testing.assert_array_equal(lib.net_model_compute(x0), want[0])
    if layers:
        y1 = co.layer1(x0)
        np.testing.assert_array_equal(lib.net_layer1(x0), y1, err_msg="layer1")
        y2 = co.layer2(y1)
        np.testing.assert_array_equal(lib.net_layer2(y1), y2, err_msg="layer2")
        y3 = co.layer3(y2)
        np.testing.assert_array_equal(lib.net_layer3(y2), y3, err_msg="layer3")
        y3t = co.layer3_flip(y3)
        np.testing.assert_array_equal(lib.net_layer3_flip_inplace(y3).ravel(), y3t.ravel(), err_msg="flip")
        y4 = co.layer4(y3t)
        np.testing.assert_array_equal(lib.net_layer4(y3t), y4, err_msg="layer4")
        np.testing.assert_array_equal(lib.net_layer5(y4), co.layer5(y4), err_msg="layer5")


@pytest.mark.parametrize("T", [480, 1125])
@pytest.mark.parametrize("N", [2, 3, 4])
@pytest.mark.parametrize("C", [8, 16, 19, 38])
def test_channel_selected_few_class(C, N, T, gpu):
    """The verdict's sweep: C in {8, 16, 19, 38} x N in {2, 3, 4} x T in {480, 1125}."""
    ps = ParamSet.synthetic(seed=1000 * C + 10 * N + T, C=C, T=T, N=N)
    _check_all_entries(ps, B=61, seed=C + N + T)
    assert not lib.params_info()["exact_division"]  # calibrated sets: the proven float requant


@pytest.mark.parametrize("C,T,N,kw", [
    (1, 64, 1, {}), (5, 100, 16, {}), (64, 513, 2, {}), (22, 960, 3, {}), (64, 960, 2, {}),
    (33, 2000, 4, {}), (64, 4096, 5, {}), (22, 1125, 2, {}), (64, 1000, 3, {}),
    (19, 480, 3, dict(reorder_bn=False)), (38, 1125, 2, dict(clip_balanced=True)),
    (16, 777, 3, dict(weight_bits=4)), (13, 640, 2, dict(stress=True)),
    (38, 480, 2, dict(stress=True, reorder_bn=False, clip_balanced=True)),
    # the time-major K-group layouts: C <= 32 uses K groups 0 and 2 (16-byte-aligned fragments at
    # C = 16, 32), 32 < C <= 64 all four (aligned at 48)
    (32, 1125, 4, {}), (17, 480, 3, {}), (24, 512, 2, {}), (31, 1000, 4, dict(reorder_bn=False)),
    (48, 960, 4, {}), (40, 1125, 3, dict(clip_balanced=True)),
])
def test_other_geometries_and_variants(C, T, N, kw, gpu):
    """Odd and extreme T (1 pooled layer-4 sample at T = 64, the 4096-sample maximum), one and
    sixteen classes, and the build variants (plain BN, balanced clipping, int4 weights, stress
    ranges) on the general kernels."""
    ps = ParamSet.synthetic(seed=C * T + N, C=C, T=T, N=N, **kw)
    _check_all_entries(ps, B=37, seed=T + N, offset=3, layers=T <= 2000)


@pytest.mark.parametrize("C,T", [(19, 1125), (38, 480)])
def test_extreme_requant_sets(C, T, gpu):
    """Factors and offsets far outside the float envelope (rails, factors up to 2^31 - 1, the fully
    suppressing REORDER_BN threshold): exact division everywhere on the general path."""
    for rb in (True, False):
        ps = ParamSet.synthetic_extreme(seed=C + T + rb, C=C, T=T, reorder_bn=rb)
        _check_all_entries(ps, B=29, seed=C, layers=True)
        assert lib.params_info()["exact_division"]


def _tile_sweep():
    """32 geometries, one per residue of layer 2's column blocks mod 32 (NB2 = ceil(T8 / 4): rest
    0 = whole 32x32 tiles, 1-16 = one or two 16x16x64 tail tiles, 17-31 = one more full tile),
    each with 0-4 full tiles, C over 1..64, N over 1..16, T mod 16 and T mod 64 varied, the
    largest trials past the LDS staging limit (unstaged fragments), and both build variants on
    some of them."""
    out = []
    for rest in range(32):
        m = max(rest % 4, 1 if rest < 2 else 0)
        T8 = 4 * (32 * m + rest) - rest % 4
        T = 8 * T8 + (3 * rest) % 8
        kw = {}
        if rest % 5 == 1:
            kw["reorder_bn"] = False
        if rest % 7 == 3:
            kw["clip_balanced"] = True
        out.append((1 + (7 * rest) % 64, T, 1 + rest % 16, kw))
    return out


@pytest.mark.parametrize("C,T,N,kw", _tile_sweep())
def test_layer2_tile_sweep(C, T, N, kw, gpu):
    """Every layer-2 tile residue (full and tail tiles), against the oracle through the batched
    time-major and channel-major entries and the single-trial net_model_compute."""
    assert 64 <= T <= 4096
    ps = ParamSet.synthetic(seed=7 * C + T + N, C=C, T=T, N=N, **kw)
    _check_all_entries(ps, B=7, seed=C * N, offset=2, layers=False)


def _random_geometries(n=256, seed=20261018):
    """n geometries drawn over the whole accepted domain (C 1..64, T 64..4096, N 1..16, both BN
    branches, both clips, int8 or int4 weights), seeded; compiled shapes drawn are kept (they run
    the general kernels only when forced, which test_compiled_geometries_forced_general covers)."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        C, T, N = int(rng.integers(1, 65)), int(rng.integers(64, 4097)), int(rng.integers(1, 17))
        if (C, T, N) in ((22, 1125, 4), (64, 1000, 4), (64, 480, 4)):
            continue
        kw = dict(reorder_bn=bool(rng.integers(0, 4)), clip_balanced=not rng.integers(0, 4),
                  weight_bits=4 if not rng.integers(0, 6) else 8)
        out.append((C, T, N, kw))
    return out


@pytest.mark.parametrize("C,T,N,kw", _random_geometries())
def test_random_geometries(C, T, N, kw, gpu):
    """Seeded draws over the accepted domain, batched time-major and channel-major and the
    single-trial entry against the oracle."""
    ps = ParamSet.synthetic(seed=C * 4099 + T * 17 + N, C=C, T=T, N=N, **kw)
    _check_all_entries(ps, B=5, seed=C + T, offset=T % 4, layers=False)


def _random_extreme(n=48, seed=31337):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        C, T, N = int(rng.integers(1, 65)), int(rng.integers(64, 4097)), int(rng.integers(1, 17))
        out.append((C, T, N, dict(reorder_bn=bool(rng.integers(0, 2)), clip_balanced=bool(rng.integers(0, 2)),
                                  mids=int(rng.choice([0, 1, 3, 11])))))
    return out


@pytest.mark.parametrize("C,T,N,kw", _random_extreme())
def test_random_extreme_sets(C, T, N, kw, gpu):
    """ParamSet.synthetic_extreme on seeded random geometries: with only constant out-of-envelope
    filters (mids = 0) the folded set runs the float kernels, with varying ones the exact-division
    kernels; both equal the oracle on the set as given."""
    ps = ParamSet.synthetic_extreme(seed=C + 131 * T + N, C=C, T=T, N=N, **kw)
    _check_all_entries(ps, B=5, seed=T, offset=1, layers=T <= 1200)
    assert lib.params_info()["exact_division"] == (kw["mids"] > 0)


def test_float_input_general(gpu):
    """net_model_compute_batch_f32 on a general geometry equals the two-pass chain (the quantiser,
    itself checked on every float32 value, then the time-major forward) and the oracle."""
    import torch

    for C, T, N in ((19, 1125, 3), (38, 480, 2), (64, 960, 4)):
        ps = ParamSet.synthetic(seed=C + T, C=C, T=T, N=N)
        lib.params_load(ps)
        g = torch.Generator(device="cuda").manual_seed(C)
        xf = torch.randn((53, C, T), dtype=torch.float32, device="cuda", generator=g) * 1.3
        xf[0, 0, :7] = torch.tensor([float("nan"), float("inf"), -float("inf"), 3.0, -3.0, 0.0, -0.0])
        q = lib.quantize_input_torch(xf, 3.0)
        want = oracle.COracle(ps).batch(q.cpu().numpy(), nthreads=NTH)
        got = lib.forward_f32_torch(xf, 3.0).cpu().numpy()
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(lib.forward_torch(q).cpu().numpy(), want)


@pytest.mark.parametrize("C,T,N,kw", _random_geometries(24, seed=4242))
def test_random_geometries_float_input(C, T, N, kw, gpu):
    """net_model_compute_batch_f32 (quantised inside the general kernel) on seeded random
    geometries: equal to the quantiser followed by the time-major forward, and to the oracle."""
    import torch

    ps = ParamSet.synthetic(seed=C + 7 * T + N, C=C, T=T, N=N, **kw)
    lib.params_load(ps)
    g = torch.Generator(device="cuda").manual_seed(T)
    xf = torch.randn((9, C, T), dtype=torch.float32, device="cuda", generator=g) * 1.7
    q = lib.quantize_input_torch(xf, 3.0)
    want = oracle.COracle(ps).batch(q.cpu().numpy(), nthreads=NTH)
    np.testing.assert_array_equal(lib.forward_f32_torch(xf, 3.0).cpu().numpy(), want)
    np.testing.assert_array_equal(lib.forward_torch(q).cpu().numpy(), want)


@pytest.mark.parametrize("C,T,wbits,rb", [(22, 1125, 8, True), (64, 1000, 8, True), (64, 480, 8, False),
                                          (22, 1125, 4, True)])
def test_compiled_geometries_forced_general(C, T, wbits, rb, gpu):
    """Both kernel families on one set: the compiled kernel and the general kernel (forced) return
    the same logits as the oracle on the compiled geometries, over a batch large enough for every
    workgroup to walk several trials."""
    import torch

    ps = ParamSet.synthetic(seed=C + T + wbits, C=C, T=T, weight_bits=wbits, reorder_bn=rb)
    rng = np.random.default_rng(T)
    B = 1537
    xp = pack_trials(rng.integers(-128, 128, size=(B, C, T)))
    xt = torch.from_numpy(xp).cuda()
    lib.params_load(ps)
    assert lib.params_info()["path"] == "float"
    y_spec = lib.forward_torch(xt).cpu().numpy()
    try:
        lib.force_general(True)
        lib.params_load(ps)
        assert lib.params_info()["path"] == "general"
        y_gen = lib.forward_torch(xt).cpu().numpy()
    finally:
        lib.force_general(False)
    np.testing.assert_array_equal(y_gen, y_spec)
    idx = np.arange(0, B, 7)
    np.testing.assert_array_equal(y_gen[idx], oracle.COracle(ps).batch(xp[idx], nthreads=NTH))


def test_general_launch_info_and_batch_limits(gpu):
    """Launch geometry of the general kernels (dynamic LDS from the dimensions) and the empty and
    one-trial batches."""
    import torch

    ps = ParamSet.synthetic(seed=3, C=38, T=960, N=2)
    lib.params_load(ps)
    info = lib.launch_info(65536)
    assert info["threads"] == 512 and info["grid"] >= 256 and 0 < info["lds_bytes"] <= 160 * 1024
    y = torch.empty((0, 2), dtype=torch.int8, device="cuda")
    lib.model_compute_batch(0, y.data_ptr(), 0)
    x = pack_trials(np.random.default_rng(0).integers(-128, 128, size=(1, 38, 960)))
    got = lib.forward_torch(torch.from_numpy(x).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.COracle(ps).batch(x))

"""Channel-major batched forward (net_model_compute_batch_ct, SURVEY §8(b)'s [B][C][T] signature).

The kernel transposes each layer-1 block through LDS itself (forward_wg.hpp, stage_block).  Its
logits must equal the time-major path's on the same trials (net_pack_trials_i8 + the batched
forward, itself oracle-checked elsewhere) and the C oracle's on a sample, for every compiled
shape and build variant, at ragged batch sizes, at any byte alignment of the input, and at the
full B = 65,536 of configs B and D.
"""
import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet

pytestmark = pytest.mark.gpu

SHAPES = [(22, 1125, 8), (64, 1000, 8), (64, 480, 8), (22, 1125, 4)]


def _packed(torch, x):
    """[B][C][T] -> the time-major batched layout [B][stride] (pad zero), on the device."""
    B, C, T = x.shape
    stride = (C * T + 15) // 16 * 16
    xp = torch.zeros((B, stride), dtype=torch.int8, device=x.device)
    xp[:, : C * T] = x.transpose(1, 2).reshape(B, C * T)
    return xp


def _ct_batch(torch, B, C, T, seed, offset=0):
    """B channel-major trials starting `offset` bytes into a fresh allocation."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    flat = torch.randint(-128, 128, (offset + B * C * T + 64,), dtype=torch.int8, device="cuda", generator=g)
    return flat[offset: offset + B * C * T].view(B, C, T)


@pytest.mark.parametrize("C,T,wbits", SHAPES, ids=["22x1125", "64x1000", "64x480", "22x1125-int4"])
@pytest.mark.parametrize("variant", ["canonical", "plain_bn", "clip_balanced"])
def test_ct_matches_time_major_and_oracle(C, T, wbits, variant, gpu):
    import torch

    ps = ParamSet.synthetic(seed=31 * C + T + wbits, C=C, T=T, weight_bits=wbits,
                            reorder_bn=variant != "plain_bn", clip_balanced=variant == "clip_balanced")
    lib.params_load(ps)
    for B, off in ((1, 0), (7, 1), (301, 3), (1000, 2)):
        x = _ct_batch(torch, B, C, T, seed=B + C, offset=off)
        y = lib.forward_ct_torch(x)
        xp = _packed(torch, x)
        want_gpu = lib.forward_torch(xp)
        torch.cuda.synchronize()
        assert torch.equal(y, want_gpu), f"B={B} offset={off}: channel-major differs from time-major"
        idx = np.unique(np.r_[0, B - 1, np.arange(0, B, max(1, B // 24))])
        want = oracle.COracle(ps).batch(xp[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
        np.testing.assert_array_equal(y.cpu().numpy()[idx], want)


def test_ct_stress_range_and_constant_inputs(gpu):
    """Stress-range parameters (both clip rails, negative truncation) and constant inputs (every
    sample at a rail): channel-major equals the oracle."""
    import torch

    C, T = 22, 1125
    ps = ParamSet.synthetic(seed=5, C=C, T=T, stress=True)
    lib.params_load(ps)
    xs = [torch.full((3, C, T), v, dtype=torch.int8, device="cuda") for v in (-128, 127, 0)]
    x = torch.cat(xs + [_ct_batch(torch, 61, C, T, seed=9)])
    y = lib.forward_ct_torch(x)
    want = oracle.COracle(ps).batch(_packed(torch, x).cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y.cpu().numpy(), want)


@pytest.mark.parametrize("C,T,wbits", [(22, 1125, 8), (22, 1125, 4), (64, 1000, 8)], ids=["B", "D", "C"])
def test_ct_full_batch(C, T, wbits, gpu):
    """B = 65,536: equal to the time-major path on every trial, deterministic, and equal to the
    oracle on 256 random trials plus the first and last 8 (whose rows meet the neighbouring trial
    or the end of the input)."""
    import torch

    B = 65536
    ps = ParamSet.synthetic(seed=77 + C + wbits, C=C, T=T, weight_bits=wbits)
    lib.params_load(ps)
    x = _ct_batch(torch, B, C, T, seed=C + 2 * wbits, offset=2)
    y = lib.forward_ct_torch(x)
    y2 = lib.forward_ct_torch(x)
    xp = _packed(torch, x)
    want_gpu = lib.forward_torch(xp)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    assert torch.equal(y, want_gpu)
    rng = np.random.default_rng(C + wbits)
    idx = np.unique(np.concatenate([rng.choice(B, 256, replace=False), np.arange(8), np.arange(B - 8, B)]))
    want = oracle.COracle(ps).batch(xp[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y.cpu().numpy()[idx], want)


def test_ct_errors(gpu):
    import torch

    ps = ParamSet.synthetic(seed=1)
    lib.params_load(ps)
    L = lib.load()
    y = torch.empty((4, 4), dtype=torch.int8, device="cuda")
    x = torch.zeros((4, 22, 1125), dtype=torch.int8, device="cuda")
    assert L.net_model_compute_batch_ct(None, y.data_ptr(), 4, 0, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_ct(x.data_ptr(), y.data_ptr() + 1, 4, 0, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_ct(x.data_ptr(), y.data_ptr(), 0, 0, None) == lib.NET_OK
    with pytest.raises(ValueError):
        lib.forward_ct_torch(torch.zeros((2, 1125, 22), dtype=torch.int8, device="cuda"))


def test_ct_graph_and_streams(gpu):
    """The channel-major entry inside a captured HIP graph (channel-major forward -> class,
    replayed over new inputs), and two launches racing on two streams (each equals the oracle)."""
    import torch

    ps = ParamSet.synthetic(seed=61)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    B, C, T = 777, 22, 1125
    rng = np.random.default_rng(61)
    xs = [rng.integers(-128, 128, size=(B, C, T)).astype(np.int8) for _ in range(3)]
    xin = torch.from_numpy(xs[0]).cuda()
    lib.forward_ct_torch(xin)  # eager call: uploads the parameters
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            logits = lib.forward_ct_torch(xin, stream=s)
            cls = lib.argmax_torch(logits, stream=s)
    for x in xs:
        xin.copy_(torch.from_numpy(x))
        g.replay()
        torch.cuda.synchronize()
        want = co.batch(_packed(torch, torch.from_numpy(x).cuda()).cpu().numpy(), nthreads=8)
        assert np.array_equal(logits.cpu().numpy(), want)
        assert np.array_equal(cls.cpu().numpy(), np.argmax(want, axis=1))
    # two streams at once, different batches
    a, b = torch.from_numpy(xs[1]).cuda(), torch.from_numpy(xs[2][:500]).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        ya = lib.forward_ct_torch(a, stream=s1)
    with torch.cuda.stream(s2):
        yb = lib.forward_ct_torch(b, stream=s2)
    torch.cuda.synchronize()
    assert np.array_equal(ya.cpu().numpy(), co.batch(_packed(torch, a).cpu().numpy(), nthreads=8))
    assert np.array_equal(yb.cpu().numpy(), co.batch(_packed(torch, b).cpu().numpy(), nthreads=8))


def test_ct_static_split(gpu):
    """Config E's static split over channel-major shards (net_model_compute_batch_multi_ct, device 0
    listed 4 times): equal to one channel-major launch over the whole batch and to the oracle at
    every shard boundary."""
    import torch
    from mibminet.shard import forward_devices, shard_bounds

    ps = ParamSet.synthetic(seed=71)
    lib.params_load(ps)
    B, C, T, world = 4099, 22, 1125, 4
    x = _ct_batch(torch, B, C, T, seed=71)
    y_split = forward_devices(x, [0] * world, channel_major=True)
    y_one = lib.forward_ct_torch(x).cpu().numpy()
    assert np.array_equal(y_split, y_one)
    edges = sorted({i for r in range(world) for lo, hi in [shard_bounds(B, world, r)] for i in (lo, hi - 1)})
    want = oracle.COracle(ps).batch(_packed(torch, x[edges]).cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y_split[edges], want)

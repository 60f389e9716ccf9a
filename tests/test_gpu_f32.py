"""Float EEG straight into the fused forward (net_model_compute_batch_f32).

Each layer-1 block is quantised inside the kernel.  The logits must equal the two-pass chain
(net_quantize_input_f32, itself checked against the NumPy restatement of the reference's
quantize_to_int in tests/test_quantize.py, then the time-major forward) on every trial, including
values on and next to every quantisation step, outside [-scale, scale], and at +-inf, for every
compiled shape and build variant, and the oracle on a sample.
"""
import numpy as np
import pytest

import oracle
from oracle import golden_np as G
from mibminet import lib
from mibminet.params import ParamSet

pytestmark = pytest.mark.gpu


def _inputs(rng, B, C, T, scale):
    x = (rng.normal(scale=0.6 * scale, size=(B, C, T))).astype(np.float32)
    # quantisation steps k * scale / 127 and their float neighbours, values past the clip, +-inf
    k = np.arange(-127, 128, dtype=np.float32)
    steps = (k * np.float32(scale) / np.float32(127)).astype(np.float32)
    special = np.concatenate([steps, np.nextafter(steps, np.float32(np.inf)), np.nextafter(steps, np.float32(-np.inf)),
                              np.array([3 * scale, -3 * scale, np.inf, -np.inf, 0.0, -0.0], np.float32)])
    flat = x.reshape(-1)
    pos = rng.choice(flat.size, size=special.size, replace=False)
    flat[pos] = special
    return x


@pytest.mark.parametrize("C,T", [(22, 1125), (64, 1000), (64, 480)])
@pytest.mark.parametrize("variant", ["canonical", "plain_bn", "clip_balanced"])
def test_f32_matches_chain(C, T, variant, gpu):
    import torch

    ps = ParamSet.synthetic(seed=C + T, C=C, T=T, reorder_bn=variant != "plain_bn",
                            clip_balanced=variant == "clip_balanced")
    lib.params_load(ps)
    rng = np.random.default_rng(C + T)
    scale = 1.7
    for B in (1, 5, 333):
        xh = _inputs(rng, B, C, T, scale)
        x = torch.from_numpy(xh).cuda()
        y = lib.forward_f32_torch(x, scale)
        want_gpu = lib.forward_torch(lib.quantize_input_torch(x, scale))
        torch.cuda.synchronize()
        assert torch.equal(y, want_gpu), f"B={B}"
    q = G.quantize_input(xh[:4], np.float32(scale))  # NumPy restatement: quantize_to_int + transpose
    want = oracle.COracle(ps).batch(q, nthreads=8)
    np.testing.assert_array_equal(y.cpu().numpy()[:4], want)


def test_f32_full_batch(gpu):
    """B = 65,536 of config B's shape from float input: equal to the two-pass chain on every trial."""
    import torch

    ps = ParamSet.synthetic(seed=91)
    lib.params_load(ps)
    g = torch.Generator(device="cuda").manual_seed(91)
    x = torch.randn((65536, 22, 1125), dtype=torch.float32, device="cuda", generator=g) * 1.2
    y = lib.forward_f32_torch(x, 2.5)
    want = lib.forward_torch(lib.quantize_input_torch(x, 2.5))
    torch.cuda.synchronize()
    assert torch.equal(y, want)


def test_f32_errors(gpu):
    import torch

    lib.params_load(ParamSet.synthetic(seed=1))
    L = lib.load()
    x = torch.zeros((4, 22, 1125), dtype=torch.float32, device="cuda")
    y = torch.empty((4, 4), dtype=torch.int8, device="cuda")
    assert L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 4, 0.0, 0, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_f32(x.data_ptr() + 2, y.data_ptr(), 3, 1.0, 0, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 0, 1.0, 0, None) == lib.NET_OK
    # outside [2^-60, 2^60] the in-kernel quotient is not proven exact
    assert L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 4, 2.0 ** -61, 0, None) == lib.NET_ERR_RANGE
    assert L.net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), 4, 2.0 ** 61, 0, None) == lib.NET_ERR_RANGE


@pytest.mark.parametrize("scale", [1.0, 3.0, 0.1, 1.7, 2.5, 200.0, 1e-3, 2.0 ** -60, 2.0 ** 60, 1.1e-18, 9.9e17])
def test_f32_quantiser_every_float(scale, gpu):
    """The in-kernel quantiser (Markstein-corrected quotient) equals the two-pass quantiser (IEEE
    division, checked against the NumPy restatement in tests/test_quantize.py) on all 2^32 float32
    bit patterns: +-0, subnormals, every normal, +-inf and every NaN."""
    import ctypes
    import torch

    L = lib.load()
    L.mibminet_test_quantize_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float,
                                              ctypes.c_int, ctypes.c_void_p]
    n = 1 << 28
    T = 1 << 14
    got = torch.empty(n, dtype=torch.int8, device="cuda")
    want = torch.empty(n, dtype=torch.int8, device="cuda")
    bad = 0
    for chunk in range(16):
        bits = torch.arange(chunk * n, (chunk + 1) * n, dtype=torch.int64, device="cuda").to(torch.int32)
        x = bits.view(torch.float32)
        assert L.mibminet_test_quantize_f32(x.data_ptr(), got.data_ptr(), n, scale, 0, None) == 0
        assert L.net_quantize_input_f32(x.data_ptr(), want.data_ptr(), n // T, 1, T, scale, 0, None) == 0
        torch.cuda.synchronize()
        diff = got != want
        if bool(diff.any()):
            i = int(torch.nonzero(diff)[0])
            bad += int(diff.sum())
            print(f"scale {scale}: bits {chunk * n + i:#010x} got {int(got[i])} want {int(want[i])}")
        del bits, x
    assert bad == 0

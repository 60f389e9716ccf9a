"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact int8.

* per-layer reference entry points (net_layer1..5, net_layer3_flip_inplace) vs the committed
  fixtures' per-layer outputs,
* net_model_compute (single trial, reference layout) vs fixture logits,
* the batched device entry point vs the C oracle on random parameters / inputs (ragged batch
  sizes, both compiled geometries, int4 weights, stress parameters),
* full BASELINE size (B = 65536): a sampled subset vs the oracle plus size-independent properties
  (determinism, permutation equivariance).
"""
import glob
import os

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "fixture_*.npz")))


def _torch():
    import torch

    assert torch.cuda.is_available(), "no HIP device"
    return torch


def run_batch(ps, x_packed, device=0):
    torch = _torch()
    lib.params_load(ps)
    xt = torch.from_numpy(np.ascontiguousarray(x_packed)).to(f"cuda:{device}")
    y = lib.forward_torch(xt)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p)[8:-4])
def test_layers_vs_fixture(path, gpu):
    f = np.load(path)
    ps = ParamSet.from_blob(f["blob"].tobytes())
    lib.params_load(ps)
    d = ps.dims
    xa = oracle.to_tc_align(f["x"][0], d.C_ALIGN)
    y1 = lib.net_layer1(xa)
    np.testing.assert_array_equal(y1, f["y1"])
    np.testing.assert_array_equal(lib.net_layer2(f["y1"]), f["y2"])
    np.testing.assert_array_equal(lib.net_layer3(f["y2"]), f["y3"])
    flipped = lib.net_layer3_flip_inplace(f["y3"])
    np.testing.assert_array_equal(flipped[: d.T8 * d.F2], f["y3t"].ravel()[: d.T8 * d.F2])
    np.testing.assert_array_equal(lib.net_layer4(f["y3t"]), f["y4"])
    np.testing.assert_array_equal(lib.net_layer5(f["y4"]), f["logits"][0])


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p)[8:-4])
def test_model_compute_vs_fixture(path, gpu):
    f = np.load(path)
    ps = ParamSet.from_blob(f["blob"].tobytes())
    lib.params_load(ps)
    for i, xi in enumerate(f["x"]):
        got = lib.net_model_compute(oracle.to_tc_align(xi, ps.dims.C_ALIGN))
        np.testing.assert_array_equal(got, f["logits"][i])
    got = run_batch(ps, pack_trials(f["x"]))
    np.testing.assert_array_equal(got, f["logits"])


@pytest.mark.parametrize("C,T,wbits,stress,B", [
    (22, 1125, 8, False, 257), (22, 1125, 8, True, 129), (22, 1125, 4, False, 300),
    (22, 1125, 4, True, 64), (64, 1000, 8, False, 200), (64, 1000, 4, True, 33),
])
def test_batch_vs_oracle_random(C, T, wbits, stress, B, gpu):
    rng = np.random.default_rng(B + C)
    for seed in range(2):
        ps = ParamSet.synthetic(seed=1000 * seed + B, C=C, T=T, weight_bits=wbits, stress=stress)
        lo, hi = (-60, 60) if seed == 0 else (-128, 128)
        x = pack_trials(rng.integers(lo, hi, size=(B, C, T)))
        want = oracle.COracle(ps).batch(x, nthreads=8)
        got = run_batch(ps, x)
        mism = np.argwhere(got != want)
        assert mism.size == 0, f"{len(mism)} mismatches, first {mism[:5].tolist()}"


def test_edge_batches(gpu):
    torch = _torch()
    ps = ParamSet.synthetic(seed=77)
    lib.params_load(ps)
    # B = 0 is a no-op
    x = torch.zeros((0, lib.trial_stride()), dtype=torch.int8, device="cuda")
    assert lib.forward_torch(x).shape == (0, 4)
    # constant inputs: zeros, both rails
    xs = np.stack([np.zeros((22, 1125)), np.full((22, 1125), 127), np.full((22, 1125), -128)]).astype(np.int8)
    want = oracle.COracle(ps).batch(pack_trials(xs))
    np.testing.assert_array_equal(run_batch(ps, pack_trials(xs)), want)
    # misaligned device pointer is rejected
    xt = torch.zeros((2, lib.trial_stride() + 1), dtype=torch.int8, device="cuda")
    with pytest.raises(lib.NetError):
        lib.model_compute_batch(xt.data_ptr() + 1, xt.data_ptr(), 1, 0)


def test_full_batch_properties(gpu):
    """B = 65536 (BASELINE config B): sampled parity, determinism, permutation equivariance."""
    torch = _torch()
    B = 65536
    ps = ParamSet.synthetic(seed=2024)
    lib.params_load(ps)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    stride = lib.trial_stride()
    x = torch.randint(-128, 128, (B, stride), dtype=torch.int8, device="cuda", generator=g)
    x[:, 22 * 1125:] = 0
    y1 = lib.forward_torch(x)
    y2 = lib.forward_torch(x)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    perm = torch.randperm(B, device="cuda", generator=g)
    y3 = lib.forward_torch(x[perm].contiguous())
    assert torch.equal(y3, y1[perm])
    idx = np.random.default_rng(0).choice(B, 512, replace=False)
    want = oracle.COracle(ps).batch(x[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y1.cpu().numpy()[idx], want)
    # every class logit takes many values (the kernel is not producing a constant)
    assert all(len(np.unique(y1[:, n].cpu().numpy())) > 10 for n in range(4))


def test_reload_params_between_calls(gpu):
    """Parameters are re-uploaded when a new blob is loaded (generation tracking)."""
    rng = np.random.default_rng(3)
    x = pack_trials(rng.integers(-128, 128, size=(16, 22, 1125)))
    for seed in (1, 2, 1):
        ps = ParamSet.synthetic(seed=seed)
        np.testing.assert_array_equal(run_batch(ps, x), oracle.COracle(ps).batch(x))


def test_batch_past_2gib(gpu):
    """B = 100,000 trials (2.48 GB of input, trial offsets past 2^31 bytes): sampled parity,
    including the batch's last trials (whose layer-1 windows run past the end of the input)."""
    torch = _torch()
    B = 100_000
    ps = ParamSet.synthetic(seed=99, stress=True)
    lib.params_load(ps)
    stride = lib.trial_stride()
    assert B * stride > 2**31
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(-128, 128, (B, stride), dtype=torch.int8, device="cuda", generator=g)
    x[:, 22 * 1125:] = 0
    y = lib.forward_torch(x)
    torch.cuda.synchronize()
    idx = np.concatenate([np.random.default_rng(1).choice(B - 64, 192, replace=False), np.arange(B - 64, B)])
    want = oracle.COracle(ps).batch(x[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y.cpu().numpy()[idx], want)

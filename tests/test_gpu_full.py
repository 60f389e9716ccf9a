"""Full-size GPU parity (BASELINE configs B, C, D at B = 65,536 and config E at B = 524,288).

The oracle cannot run a whole batch in seconds, so each test combines
* a sampled oracle comparison (random trials plus the batch's / every shard's first and last
  trials, whose layer-1 windows meet the neighbouring trial or the end of the input),
* size-independent properties: determinism across launches and trial-permutation equivariance,
* for config E, equality of the static 8-way split (net_model_compute_batch_multi)
  with one launch over the whole batch.
"""
import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet
from mibminet.shard import forward_devices, shard_bounds

pytestmark = pytest.mark.gpu


def _batch(torch, B, C, T, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randint(-128, 128, (B, lib.trial_stride()), dtype=torch.int8, device="cuda", generator=g)
    x[:, C * T:] = 0
    return x, g


def _sampled_oracle(ps, x, y, idx):
    import torch

    want = oracle.COracle(ps).batch(x[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
    np.testing.assert_array_equal(y[idx], want)


@pytest.mark.parametrize("C,T,wbits", [(22, 1125, 8), (64, 1000, 8), (22, 1125, 4)], ids=["B", "C", "D"])
def test_full_batch_configs(C, T, wbits, gpu):
    """B = 65,536 of config B (22 x 1125), C (64 x 1000) and D (int4 weights): sampled parity
    (512 random trials and the first/last 16), determinism, permutation equivariance."""
    import torch

    B = 65536
    ps = ParamSet.synthetic(seed=2024 + C + wbits, C=C, T=T, weight_bits=wbits)
    lib.params_load(ps)
    x, g = _batch(torch, B, C, T, seed=C + wbits)
    y1 = lib.forward_torch(x)
    y2 = lib.forward_torch(x)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    perm = torch.randperm(B, device="cuda", generator=g)
    y3 = lib.forward_torch(x[perm].contiguous())
    assert torch.equal(y3, y1[perm])
    del y3
    yh = y1.cpu().numpy()
    rng = np.random.default_rng(C * 10 + wbits)
    idx = np.unique(np.concatenate([rng.choice(B, 512, replace=False), np.arange(16), np.arange(B - 16, B)]))
    _sampled_oracle(ps, x, yh, idx)
    assert all(len(np.unique(yh[:, n])) > 10 for n in range(4))


def test_config_e_static_split(gpu):
    """Config E: 524,288 trials static-split 8 ways (65,536 per shard; device 0 listed 8 times
    stands in for the 8-GPU node).  The split equals one launch over the whole batch, is
    deterministic, and matches the oracle on 512 random trials plus the first and last 8 trials
    of every shard."""
    import torch

    B, world = 524288, 8
    ps = ParamSet.synthetic(seed=524288)
    lib.params_load(ps)
    x, _ = _batch(torch, B, 22, 1125, seed=8)
    devices = [0] * world
    y_split = forward_devices(x, devices)
    assert y_split.shape == (B, 4)
    y_split2 = forward_devices(x, devices)
    assert np.array_equal(y_split, y_split2)
    y_one = lib.forward_torch(x)
    torch.cuda.synchronize()
    assert np.array_equal(y_split, y_one.cpu().numpy())
    del y_one
    edges = []
    for r in range(world):
        lo, hi = shard_bounds(B, world, r)
        assert hi - lo == 65536
        edges += list(range(lo, lo + 8)) + list(range(hi - 8, hi))
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([rng.choice(B, 512, replace=False), np.array(edges)]))
    _sampled_oracle(ps, x, y_split, idx)

"""Parameter fuzz at the full shapes: many seeded networks (calibrated and stress-range factors
and offsets, both BN branches, both clip modes, int8 and int4 weights), each run on a batch of
trials with the reference tests' input range (randint(-60, 60), model/testcase.py:53) and the
full int8 range, compared bit for bit with the C oracle."""
import os

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu


def _cases():
    out = []
    for seed in range(24):
        C, T = (64, 1000) if seed % 4 == 3 else (64, 480) if seed % 8 == 5 else (22, 1125)
        out.append(dict(seed=100 + seed, C=C, T=T, stress=bool(seed % 2), rb=seed % 3 != 2,
                        cb=seed % 5 == 4, wbits=4 if seed % 7 == 6 else 8))
    return out


@pytest.mark.parametrize("case", _cases(), ids=lambda c: "s{seed}-{C}x{T}-st{stress:d}-rb{rb:d}-cb{cb:d}-w{wbits}".format(**c))
def test_fuzz_vs_oracle(gpu, case):
    import torch

    ps = ParamSet.synthetic(seed=case["seed"], C=case["C"], T=case["T"], weight_bits=case["wbits"],
                            stress=case["stress"], reorder_bn=case["rb"], clip_balanced=case["cb"])
    lib.params_load(ps)
    rng = np.random.default_rng(case["seed"])
    B = 96
    lo, hi = (-60, 60) if case["seed"] % 2 else (-128, 128)
    x = pack_trials(rng.integers(lo, hi, size=(B, case["C"], case["T"])))
    got = lib.forward_torch(torch.from_numpy(x).cuda()).cpu().numpy()
    want = oracle.COracle(ps).batch(x, nthreads=min(16, os.cpu_count() or 1))
    assert np.array_equal(got, want)


def _edge_net(seed, C=22, T=1125):
    """Offsets within one of the exact-requant envelope's edges and extreme
    factors (±1, small primes, 2^20 + 7, negative BN scales)."""
    ps = ParamSet.synthetic(seed=seed, C=C, T=T, stress=True)
    rng = np.random.default_rng(seed)
    A = 128 * 128
    b1, b2, b4 = (1 << 22) - C * A - 1, (1 << 24) - 8 * 64 * A - 1, (1 << 24) - 8 * 16 * A - 1
    facs = np.array([1, -1, 2, 3, -7, 255, 65537, (1 << 20) + 7, -(1 << 20) - 9, 31, -127, 1 << 16], np.int64)
    for name, b in (("l1", b1), ("l2", b2), ("l4", b4)):
        off = rng.integers(-b, b + 1, size=16)
        off[:4] = [b, -b, b - 1, -(b - 1)]
        getattr(ps, f"{name}_offset")[:] = off.astype(np.int32)
        getattr(ps, f"{name}_factor")[:] = rng.choice(facs, size=16).astype(np.int32)
    ps.l3_factor = int(rng.choice([1, -1, 3, 1 << 20]))
    ps.l5_factor = int(rng.choice([1, -2, 5, 1 << 20]))
    return ps


@pytest.mark.parametrize("seed,C,T", [(1, 22, 1125), (2, 22, 1125), (3, 64, 1000), (4, 22, 1125), (5, 64, 480)])
def test_envelope_edges_vs_oracle(gpu, seed, C, T):
    import torch

    ps = _edge_net(seed, C, T)
    lib.params_load(ps)
    rng = np.random.default_rng(seed)
    x = pack_trials(rng.integers(-128, 128, size=(128, C, T)))
    got = lib.forward_torch(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle.COracle(ps).batch(x, nthreads=min(16, os.cpu_count() or 1)))

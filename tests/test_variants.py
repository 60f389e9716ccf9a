"""Build variants of the reference forward: the plain BN branches that the
reference compiles without -DREORDER_BN (layer2.c:139-210, layer4.c:91-133), covered by its own
model test matrix (test/cl/net/model/testcase.py:74-80, reorder False/True).

CPU: the C restatement (oracle.c) and the NumPy golden-model restatement agree on the plain
branch, and the one place where the reference's C and golden model differ (layer 4 of the plain
branch: the C does not clip each element to int8 before the ReLU, golden_model.py:337-340 does)
is pinned explicitly.  GPU: the HIP path against the C oracle, per layer and batched, both
geometries, bit-exact.
"""
import numpy as np
import pytest

import oracle
from oracle import golden_np as G
from mibminet.params import ParamSet, pack_trials


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_plain_branch_c_vs_golden(seed):
    ps = ParamSet.synthetic(seed=seed, C=8, T=512, reorder_bn=False)
    rng = np.random.default_rng(seed)
    x = rng.integers(-60, 60, size=(5, 8, 512))
    assert np.array_equal(oracle.COracle(ps).batch(pack_trials(x), nthreads=2), G.forward(ps, x))


def test_plain_blob_roundtrip():
    ps = ParamSet.synthetic(seed=4, reorder_bn=False)
    back = ParamSet.from_blob(ps.to_blob())
    assert back.reorder_bn is False
    assert ParamSet.from_blob(ParamSet.synthetic(seed=4).to_blob()).reorder_bn is True


def test_plain_layer4_c_does_not_clip_elements():
    """A window whose first element exceeds 127: the C (layer4.c:113-118) sums it unclipped, the
    golden model clips it to 127 first.  The oracle and the GPU path follow the C."""
    ps = ParamSet.synthetic(seed=9, C=8, T=512, reorder_bn=False)
    ps.l4_factor[:] = 8  # factor >> 3 == 1: element = dot + (offset >> 3)
    ps.l4_offset[:] = 0
    d = ps.dims
    y3t = np.zeros((d.T8, d.F2), np.int8)
    y3t[0, :] = 1  # window 0: element 0 = row sum of W4, elements 1..7 = 0
    el = ps.l4_weight.astype(np.int64).sum(1)
    y4 = oracle.COracle(ps).layer4(y3t)
    want_c = np.clip(np.maximum(el, 0) >> 3, -128, 127)
    want_golden = np.clip(np.maximum(np.clip(el, -128, 127), 0) >> 3, -128, 127)
    assert np.array_equal(y4[:, 0], want_c.astype(np.int8))
    assert np.any(want_c != want_golden), "test data must exercise the difference"
    # the NumPy golden restatement keeps the golden model's behaviour
    g = G.layer4(ps, y3t.T[None].astype(np.int64))
    assert np.array_equal(g[0][:, 0], want_golden)


def _run(ps, x):
    import torch
    from mibminet import lib

    lib.params_load(ps)
    return lib.forward_torch(torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")).cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("C,T,wbits,stress,B", [
    (22, 1125, 8, False, 515), (22, 1125, 4, False, 200), (22, 1125, 8, True, 300), (64, 1000, 8, False, 257),
])
def test_gpu_plain_branch_batch(gpu, C, T, wbits, stress, B):
    ps = ParamSet.synthetic(seed=C + B, C=C, T=T, weight_bits=wbits, stress=stress, reorder_bn=False)
    rng = np.random.default_rng(B)
    x = pack_trials(rng.integers(-128, 128, size=(B, C, T)))
    assert np.array_equal(_run(ps, x), oracle.COracle(ps).batch(x, nthreads=8))


@pytest.mark.gpu
def test_gpu_plain_branch_layers(gpu):
    from mibminet import lib

    ps = ParamSet.synthetic(seed=21, reorder_bn=False)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    d = ps.dims
    rng = np.random.default_rng(21)
    x = oracle.to_tc_align(rng.integers(-100, 100, size=(d.C, d.T)), d.C_ALIGN)
    y1 = co.layer1(x)
    y2 = co.layer2(y1)
    assert np.array_equal(lib.net_layer2(y1), y2)
    y3 = co.layer3(y2)
    y3t = co.layer3_flip(y3)
    assert np.array_equal(lib.net_layer4(y3t), co.layer4(y3t))
    # a window with an element far above 127 (the C semantics, see the CPU test above)
    big = np.zeros_like(y3t)
    big.reshape(-1)[: d.F2] = 127
    assert np.array_equal(lib.net_layer4(big), co.layer4(big))
    assert np.array_equal(lib.net_model_compute(x), co.model(x))

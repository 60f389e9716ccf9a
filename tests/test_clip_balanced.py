"""The golden model's clip_balanced=True mode: every requantised output
clips to [-127, 127] instead of [-128, 127] (python_utils/functional.py:89-91, used by all five
layers of golden_model.py:195-378).  The reference C has no such build (__CLIP_R(x, 127) clips to
-128) and its own tests pass clip_balanced=False (test/cl/net/model/testcase.py:51), so this mode
is pinned by the golden model alone: the NumPy restatement (golden_np) and the C restatement
(oracle.c, clip_lo = -127) must agree, and the HIP path must equal them bit for bit.

The blob carries the mode as flag bit 1 (ParamSet.clip_balanced).
"""
import struct

import numpy as np
import pytest

import oracle
from oracle import golden_np as G
from mibminet import lib
from mibminet.params import FLAG_CLIP_BALANCED, HEADER_FMT, ParamSet, pack_trials


def test_blob_roundtrip_and_flags():
    for rb in (True, False):
        ps = ParamSet.synthetic(seed=3, reorder_bn=rb, clip_balanced=True)
        back = ParamSet.from_blob(ps.to_blob())
        assert back.clip_balanced is True and back.reorder_bn is rb
        assert back.flags & FLAG_CLIP_BALANCED
    assert ParamSet.from_blob(ParamSet.synthetic(seed=3).to_blob()).clip_balanced is False


def _with_flags(blob, flags):
    head = list(struct.unpack_from(HEADER_FMT, blob, 0))
    head[-1] = flags
    return struct.pack(HEADER_FMT, *head) + blob[struct.calcsize(HEADER_FMT):]


def test_unknown_flags_rejected():
    blob = _with_flags(ParamSet.synthetic(seed=3).to_blob(), 1 | 4)
    with pytest.raises(ValueError):
        ParamSet.from_blob(blob)
    L = lib.load()
    assert L.net_params_load(blob, len(blob)) == lib.NET_ERR_BLOB
    ok = _with_flags(blob, 1 | 2)
    assert L.net_params_load(ok, len(ok)) == 0
    lib.params_unload()


@pytest.mark.parametrize("rb", [True, False])
@pytest.mark.parametrize("seed", [0, 1])
def test_c_vs_golden_balanced(rb, seed):
    """Stress parameters saturate often, so -128 occurs in the unbalanced run.  The plain branch
    uses the calibrated parameters and the reference tests' input range: otherwise its layer 4 reaches the one place where the
    C and the golden model differ (test_variants.py), which is not what this test is about."""
    def net(cb):
        p = ParamSet.synthetic(seed=seed, C=8, T=512, stress=rb, reorder_bn=rb, clip_balanced=cb)
        if not rb:  # push four layer-1 filters onto the lower rail
            p.l1_offset[:4] -= 100 * np.abs(p.l1_factor[:4])
        return p

    ps = net(True)
    rng = np.random.default_rng(seed)
    x = rng.integers(-128, 128, size=(6, 8, 512)) if rb else rng.integers(-60, 60, size=(6, 8, 512))
    z, inter = G.forward(ps, x, return_all=True)
    assert np.array_equal(oracle.COracle(ps).batch(pack_trials(x), nthreads=2), z)
    for y in (z,) + tuple(inter):
        assert y.min() >= -127
    # the same network unbalanced reaches -128 somewhere: the test exercises the difference
    pu = net(False)
    zu, interu = G.forward(pu, x, return_all=True)
    assert any((y == -128).any() for y in (zu,) + tuple(interu))
    assert np.array_equal(oracle.COracle(pu).batch(pack_trials(x), nthreads=2), zu)


def test_c_layers_balanced():
    """Per-layer: each C layer equals the golden layer on the same (balanced) input."""
    ps = ParamSet.synthetic(seed=5, C=8, T=512, stress=True, clip_balanced=True)
    co = oracle.COracle(ps)
    d = ps.dims
    rng = np.random.default_rng(5)
    x = rng.integers(-128, 128, size=(d.C, d.T))
    _, (g1, g2, g3, g4) = G.forward(ps, x, return_all=True)
    y1 = co.layer1(oracle.to_tc_align(x, d.C_ALIGN))
    assert np.array_equal(y1[:, : d.T], g1)
    y2 = co.layer2(y1)
    assert np.array_equal(y2[:, : d.T8], g2)
    y3 = co.layer3(y2)
    assert np.array_equal(y3[:, : d.T8], g3)


@pytest.mark.gpu
@pytest.mark.parametrize("C,T,rb,B", [
    (22, 1125, True, 515), (22, 1125, False, 300), (64, 1000, True, 257), (64, 1000, False, 130),
])
def test_gpu_balanced_batch(gpu, C, T, rb, B):
    import torch

    for stress in (True, False):
        ps = ParamSet.synthetic(seed=C + B, C=C, T=T, stress=stress, reorder_bn=rb, clip_balanced=True)
        rng = np.random.default_rng(B)
        x = pack_trials(rng.integers(-128, 128, size=(B, C, T)))
        lib.params_load(ps)
        got = lib.forward_torch(torch.from_numpy(x).to("cuda:0")).cpu().numpy()
        assert np.array_equal(got, oracle.COracle(ps).batch(x, nthreads=8)), f"stress={stress}"
        assert got.min() >= -127


@pytest.mark.gpu
@pytest.mark.parametrize("C,T", [(22, 1125), (64, 1000)])
def test_gpu_balanced_layers(gpu, C, T):
    ps = ParamSet.synthetic(seed=31, C=C, T=T, stress=True, clip_balanced=True)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    d = ps.dims
    rng = np.random.default_rng(31)
    x = oracle.to_tc_align(rng.integers(-128, 128, size=(d.C, d.T)), d.C_ALIGN)
    y1 = co.layer1(x)
    assert np.array_equal(lib.net_layer1(x), y1)
    y2 = co.layer2(y1)
    assert np.array_equal(lib.net_layer2(y1), y2)
    y3 = co.layer3(y2)
    assert np.array_equal(lib.net_layer3(y2), y3)
    y3t = co.layer3_flip(y3)
    y4 = co.layer4(y3t)
    assert np.array_equal(lib.net_layer4(y3t), y4)
    assert np.array_equal(lib.net_layer5(y4), co.layer5(y4))
    assert np.array_equal(lib.net_model_compute(x), co.model(x))

"""The third compiled geometry: 64 channels x 480 samples, the reference's PhysioNet MMMI
edgeEEGNet (QuantLab/PhysionetMMMI/config_INQ.json: F1 = F2 = 16, D = 1, C = 64, T = 480, N = 4).
Its 60 pooled layer-2 samples per filter fill half of one 32x32 tile, which the kernel computes
as a partial tile (Cfg::MT / TB, forward_wg.hpp).  Per layer and batched against the oracle."""
import os

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu
C, T = 64, 480


@pytest.mark.parametrize("rb,cb,stress,wbits,B", [
    (True, False, False, 8, 1000), (True, False, True, 8, 777), (False, False, False, 8, 300),
    (True, True, True, 8, 200), (True, False, False, 4, 130), (True, False, False, 8, 1),
])
def test_batch_64x480(gpu, rb, cb, stress, wbits, B):
    import torch

    ps = ParamSet.synthetic(seed=B, C=C, T=T, weight_bits=wbits, stress=stress, reorder_bn=rb, clip_balanced=cb)
    lib.params_load(ps)
    assert lib.trial_stride() == C * T
    rng = np.random.default_rng(B)
    x = pack_trials(rng.integers(-128, 128, size=(B, C, T)))
    got = lib.forward_torch(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.array_equal(got, oracle.COracle(ps).batch(x, nthreads=min(16, os.cpu_count() or 1)))


@pytest.mark.parametrize("stress", [False, True])
def test_layers_64x480(gpu, stress):
    ps = ParamSet.synthetic(seed=480 + stress, C=C, T=T, stress=stress)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    d = ps.dims
    rng = np.random.default_rng(480)
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

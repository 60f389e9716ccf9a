"""Oracle pinning (CPU): the C restatement (oracle/oracle.c) and the NumPy restatement of the
golden model (oracle/golden_np.py) against the reference's known answer and each other."""
import glob
import json
import os

import numpy as np
import pytest

import oracle
from mibminet.params import ParamSet, appendix_b_net

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_appendix_b_known_answer():
    """reference golden model output on the seed-0 synthetic export."""
    kat = json.load(open(os.path.join(GOLDEN, "appendix_b.json")))
    net, cfg, x = appendix_b_net(0)
    ps = ParamSet.from_quantlab(net, cfg)
    assert ps.l1_factor[:4].tolist() == kat["l1_factor_head"]
    assert ps.l1_offset[:4].tolist() == kat["l1_offset_head"]
    assert ps.l2_factor[:4].tolist() == kat["l2_factor_head"]
    assert ps.l2_offset[:4].tolist() == kat["l2_offset_head"]
    assert ps.l3_factor == kat["l3_factor"]
    assert ps.l4_factor[:4].tolist() == kat["l4_factor_head"]
    assert ps.l4_offset[:4].tolist() == kat["l4_offset_head"]
    assert ps.l5_factor == kat["l5_factor"]
    assert ps.l5_bias.tolist() == kat["l5_bias"]
    assert oracle.golden_np.forward(ps, x).tolist() == kat["logits"]
    co = oracle.COracle(ps)
    assert co.model(oracle.to_tc_align(x.astype(np.int8), ps.dims.C_ALIGN)).tolist() == kat["logits"]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "fixture_*.npz"))))
def test_fixture(path):
    f = np.load(path)
    ps = ParamSet.from_blob(f["blob"].tobytes())
    d = ps.dims
    co = oracle.COracle(ps)
    x = f["x"]
    got = np.stack([co.model(oracle.to_tc_align(xi, d.C_ALIGN)) for xi in x])
    assert np.array_equal(got, f["logits"])
    if ps.reorder_bn:  # plain BN: the golden model clips layer-4 elements, the C does not (layers 1-3 below)
        assert np.array_equal(oracle.golden_np.forward(ps, x), f["logits"].astype(np.int64))
    xa = oracle.to_tc_align(x[0], d.C_ALIGN)
    y1 = co.layer1(xa)
    assert np.array_equal(y1, f["y1"])
    assert np.array_equal(co.layer2(f["y1"]), f["y2"])
    assert np.array_equal(co.layer3(f["y2"]), f["y3"])
    assert np.array_equal(co.layer3_flip(f["y3"]), f["y3t"])
    assert np.array_equal(co.layer4(f["y3t"]), f["y4"])
    assert np.array_equal(co.layer5(f["y4"]), f["logits"][0])
    # per-layer agreement with the golden-model restatement
    g = oracle.golden_np
    gy1 = g.layer1(ps, x[:1].astype(np.int64))
    assert np.array_equal(gy1[0], f["y1"][:, : d.T])
    gy2 = g.layer2(ps, gy1)
    assert np.array_equal(gy2[0], f["y2"][:, : d.T8])
    gy3 = g.layer3(ps, gy2)
    assert np.array_equal(gy3[0], f["y3"][:, : d.T8])
    if ps.reorder_bn:
        gy4 = g.layer4(ps, gy3)
        assert np.array_equal(gy4[0], f["y4"][:, : d.T64])


@pytest.mark.parametrize("C,T,wbits,stress", [(22, 1125, 8, False), (22, 1125, 8, True),
                                              (64, 1000, 8, False), (22, 1125, 4, False),
                                              (22, 1125, 4, True), (8, 512, 8, False)])
def test_c_vs_numpy_random(C, T, wbits, stress):
    rng = np.random.default_rng(C * 1000 + T + wbits + stress)
    for seed in range(3):
        ps = ParamSet.synthetic(seed=100 + seed, C=C, T=T, weight_bits=wbits, stress=stress)
        x = rng.integers(-128, 128, size=(5, C, T))
        from mibminet.params import pack_trials
        got = oracle.COracle(ps).batch(pack_trials(x), nthreads=2)
        want = oracle.golden_np.forward(ps, x)
        assert np.array_equal(got.astype(np.int64), want)


def test_batch_driver_matches_single():
    ps = ParamSet.synthetic(seed=5)
    rng = np.random.default_rng(5)
    x = rng.integers(-128, 128, size=(9, 22, 1125))
    from mibminet.params import pack_trials
    co = oracle.COracle(ps)
    b1 = co.batch(pack_trials(x), nthreads=1)
    b4 = co.batch(pack_trials(x), nthreads=4)
    single = np.stack([co.model(oracle.to_tc_align(xi, 24)) for xi in x.astype(np.int8)])
    assert np.array_equal(b1, single) and np.array_equal(b4, single)

"""Generates the committed parity fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_fixtures.py``).

Each ``fixture_*.npz`` holds a parameter blob (``blob``, uint8), int8 inputs ``x`` [n][C][T], the
expected logits ``logits`` [n][N] and trial 0's per-layer outputs in the reference layouts
(``y1`` [F1][T_ALIGN], ``y2`` [F2][T8_ALIGN], ``y3`` [F2][T8_ALIGN], ``y3t`` [T8][F2] after the
flip, ``y4`` [F2][T64_ALIGN]).  Expected values come from the C oracle and are cross-checked
against the NumPy golden-model restatement before writing; the oracle itself is pinned by the
reference's known answer in ``appendix_b.json``.

The reference ships no vectors of its own (data/*.npz are git-ignored upstream), so these
fixtures pin the *restatement*; the pin to the reference is the Appendix B known answer.
"""
import argparse
import io
import os
import sys
import zipfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from mibminet.params import ParamSet, appendix_b_net  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def save_npz(path, **arrays):
    """np.savez_compressed with fixed member timestamps and order, so that regenerating a fixture
    gives the committed file byte for byte (tests/test_fixtures.py checks it)."""
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as z:
        for name, a in arrays.items():
            buf = io.BytesIO()
            np.lib.format.write_array(buf, np.asanyarray(a), allow_pickle=False)
            info = zipfile.ZipInfo(name + ".npy", date_time=(1980, 1, 1, 0, 0, 0))
            info.compress_type = zipfile.ZIP_DEFLATED
            info.external_attr = 0o644 << 16
            z.writestr(info, buf.getvalue())


def make(name, ps, x, out=OUT, golden=True):
    """golden=False for the plain-BN build: there the golden model clips each layer-4 element and
    the C does not (golden_np.py, layer4), and these fixtures follow the C; its layers 1-3 are still
    cross-checked against the golden restatement on trial 0."""
    d = ps.dims
    co = oracle.COracle(ps)
    logits = np.stack([co.model(oracle.to_tc_align(xi, d.C_ALIGN)) for xi in x])
    if golden:
        ref = oracle.golden_np.forward(ps, x)
        assert np.array_equal(logits.astype(np.int64), ref), name
    else:
        _, (g1, g2, g3, _) = oracle.golden_np.forward(ps, x[0], return_all=True)
        yy = co.layer1(oracle.to_tc_align(x[0], d.C_ALIGN))
        assert np.array_equal(yy[:, : d.T], g1), name
        yy = co.layer2(yy)
        assert np.array_equal(yy[:, : d.T8], g2), name
        yy = co.layer3(yy)
        assert np.array_equal(yy[:, : d.T8], g3), name
    xa = oracle.to_tc_align(x[0], d.C_ALIGN)
    y1 = co.layer1(xa)
    y2 = co.layer2(y1)
    y3 = co.layer3(y2)
    y3t = co.layer3_flip(y3)
    y4 = co.layer4(y3t)
    save_npz(os.path.join(out, f"fixture_{name}.npz"),
             blob=np.frombuffer(ps.to_blob(), np.uint8), x=x.astype(np.int8),
             logits=logits, y1=y1, y2=y2, y3=y3, y3t=y3t, y4=y4)
    print(name, logits.tolist()[:3])


def main(out=OUT):
    rng = np.random.default_rng(20250328)
    # config B (22 x 1125), calibrated synthetic parameters, reference test input distribution
    ps = ParamSet.synthetic(seed=11, C=22, T=1125)
    x = rng.integers(-60, 60, size=(6, 22, 1125))
    x[1] = rng.integers(-128, 128, size=(22, 1125))     # full int8 range
    x[2] = 127
    x[3] = -128
    make("b22", ps, x, out=out)
    # config B with the literal SURVEY §8(d) stress ranges (rails, negative truncation)
    ps = ParamSet.synthetic(seed=12, C=22, T=1125, stress=True)
    make("b22_stress", ps, rng.integers(-128, 128, size=(4, 22, 1125)), out=out)
    # config C (64 x 1000)
    ps = ParamSet.synthetic(seed=13, C=64, T=1000)
    make("c64", ps, rng.integers(-60, 60, size=(3, 64, 1000)), out=out)
    # config D (22 x 1125, int4 weights)
    ps = ParamSet.synthetic(seed=14, C=22, T=1125, weight_bits=4)
    make("d22_int4", ps, rng.integers(-128, 128, size=(4, 22, 1125)), out=out)
    # Appendix B parameters (converted from the float QuantLab-style export) with
    # the reference model test's input distribution (test/cl/net/model/testcase.py:53)
    net, cfg, x0 = appendix_b_net(0)
    ps = ParamSet.from_quantlab(net, cfg)
    x = np.concatenate([x0[None], rng.integers(-60, 60, size=(3, 22, 1125))])
    make("appb", ps, x, out=out)
    # config B's shape with factors and offsets far outside the float requant envelope (offsets
    # near +-2^30, factors 1 and +-(2^31 - 1), threshold-suppressed filters, |offsets| past 2^22):
    # the exact-division kernels (Cfg::XR); full int8 range and the reference test range
    ps = ParamSet.synthetic_extreme(seed=15, C=22, T=1125)
    x = rng.integers(-128, 128, size=(5, 22, 1125))
    x[3:] = rng.integers(-60, 60, size=(2, 22, 1125))
    make("xr22", ps, x, out=out)
    # the plain-BN build (no -DREORDER_BN, layer2.c:139-210 / layer4.c:113-130): calibrated
    # parameters, then an extreme set on its exact-division kernels
    ps = ParamSet.synthetic(seed=16, C=22, T=1125, reorder_bn=False)
    x = rng.integers(-128, 128, size=(4, 22, 1125))
    x[2:] = rng.integers(-60, 60, size=(2, 22, 1125))
    make("b22_plain", ps, x, out=out, golden=False)
    ps = ParamSet.synthetic_extreme(seed=17, C=22, T=1125, reorder_bn=False)
    make("xr22_plain", ps, rng.integers(-128, 128, size=(4, 22, 1125)), out=out, golden=False)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=OUT, help="output directory (default: tests/golden)")
    main(ap.parse_args().out)

"""The step after the path: class per trial and the accuracy harness on a
``benchmark.npz`` laid out as QuantLab/export_net_data.py:89-101 writes it.  The reference ships
no data set, so the files here are synthetic (same keys, shapes and dtypes).

CPU: the loader and the C ABI's argument checks.  GPU: net_argmax_batch against np.argmax (first
maximal index, as torch.max(dim=1) in QuantLab's postprocess.py:6-8) on tie-heavy logits, and
the whole harness (GPU quantiser -> fused forward -> argmax) against the oracle chain
(golden_np.quantize_input -> oracle.c forward -> np.argmax).
"""
import json

import numpy as np
import pytest

import oracle
from oracle import golden_np as G
from mibminet import evaluate as E
from mibminet import lib
from mibminet.params import ParamSet, appendix_b_net, ste_quant


def _signals(rng, n, C, T):
    """Per-channel sinusoids of random frequency, phase and amplitude plus noise: unlike pure
    noise, these move the synthetic networks' logits enough to give several classes."""
    t = np.arange(T)
    f = rng.uniform(0.002, 0.05, (n, C, 1))
    ph = rng.uniform(0, 2 * np.pi, (n, C, 1))
    amp = rng.uniform(0, 3, (n, C, 1))
    return (amp * np.sin(2 * np.pi * f * t + ph) + rng.normal(0, 0.3, (n, C, T))).astype(np.float32)


def _write_benchmark(path, n, C, T, N, seed, with_pred=True):
    """Lists of per-trial arrays, as export_net_data.py:92-101 collects and saves them."""
    rng = np.random.default_rng(seed)
    samples = list(_signals(rng, n, C, T)[:, None, None])
    labels = [np.array(rng.integers(0, N)) for _ in range(n)]
    kw = dict(samples=samples, labels=labels)
    if with_pred:
        kw["predictions"] = [rng.normal(size=(1, N)).astype(np.float32) for _ in range(n)]
    np.savez(path, **kw)


def test_load_benchmark(tmp_path):
    p = str(tmp_path / "benchmark.npz")
    _write_benchmark(p, 7, 22, 1125, 4, 0)
    s, y, pr = E.load_benchmark(p)
    assert s.shape == (7, 22, 1125) and s.dtype == np.float32 and s.flags.c_contiguous
    assert y.shape == (7,) and y.dtype == np.int64
    assert pr.shape == (7, 4)
    p2 = str(tmp_path / "nopred.npz")
    _write_benchmark(p2, 3, 8, 512, 4, 1, with_pred=False)
    s2, _, pr2 = E.load_benchmark(p2)
    assert s2.shape == (3, 8, 512) and pr2 is None
    p3 = str(tmp_path / "bad.npz")
    np.savez(p3, samples=np.zeros((3, 1, 1, 8, 512), np.float32), labels=np.zeros(2))
    with pytest.raises(ValueError):
        E.load_benchmark(p3)


def test_argmax_abi_checks():
    L = lib.load()
    assert L.net_argmax_batch(None, None, 0, 4, 0, None) == 0  # empty batch: nothing to do
    assert L.net_argmax_batch(None, None, 1, 4, 0, None) == lib.NET_ERR_INVALID
    buf = (np.zeros(8, np.int8), np.zeros(2, np.int32))
    assert L.net_argmax_batch(buf[0].ctypes.data, buf[1].ctypes.data, 2, 0, 0, None) == lib.NET_ERR_INVALID
    assert L.net_argmax_batch(buf[0].ctypes.data, buf[1].ctypes.data, 2, 65, 0, None) == lib.NET_ERR_INVALID
    # int trial indices in the kernels: B past INT32_MAX - 4 * 256 is rejected before any launch
    assert L.net_argmax_batch(buf[0].ctypes.data, buf[1].ctypes.data, 2**31 - 1024, 4, 0, None) == lib.NET_ERR_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("N,B", [(4, 100_003), (7, 1_000), (1, 33)])
def test_gpu_argmax_first_max(gpu, N, B):
    import torch

    rng = np.random.default_rng(N + B)
    z = rng.choice(np.array([-128, -1, 0, 5, 127], np.int8), size=(B, N))  # many ties
    got = lib.argmax_torch(torch.from_numpy(z).to("cuda:0")).cpu().numpy()
    assert np.array_equal(got, np.argmax(z, axis=1))
    assert np.array_equal(got, torch.max(torch.from_numpy(z).to(torch.int32), dim=1).indices.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 1, 2, 3])
def test_gpu_argmax4_alignment(gpu, shift):
    """N = 4 takes four trials per thread when both buffers are 16-byte aligned (k_argmax4) and the
    per-trial kernel otherwise; logits and classes starting `shift` trials into their buffers
    cover both paths and every tail length."""
    import torch

    B = 4099
    rng = np.random.default_rng(40 + shift)
    z = rng.choice(np.array([-128, -1, 0, 5, 127], np.int8), size=(B + shift, 4))
    zd = torch.from_numpy(z).to("cuda:0")
    out = torch.full((B + shift,), -1, dtype=torch.int32, device="cuda:0")
    L = lib.load()
    rc = L.net_argmax_batch(zd.data_ptr() + 4 * shift, out.data_ptr() + 4 * shift, B, 4, 0, None)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got[shift:], np.argmax(z[shift:], axis=1))
    assert (got[:shift] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("clip_balanced", [False, True])
def test_gpu_harness_vs_oracle(gpu, tmp_path, clip_balanced):
    bench = str(tmp_path / "benchmark.npz")
    _write_benchmark(bench, 300, 22, 1125, 4, 5)
    samples, labels, pred = E.load_benchmark(bench)
    ps = ParamSet.synthetic(seed=2, clip_balanced=clip_balanced)
    scale = np.float32(2.0)
    # oracle chain
    xq = G.quantize_input(samples, scale)
    logits = oracle.COracle(ps).batch(xq, nthreads=8)
    want = np.argmax(logits, axis=1)
    assert len(np.unique(want)) >= 2, "the synthetic set must not collapse onto one class"
    cls, lg = E.classify(ps, samples, scale)
    assert np.array_equal(lg.cpu().numpy(), logits)
    assert np.array_equal(cls.cpu().numpy(), want)
    res = E.evaluate(ps, samples, labels, scale, pred)
    assert res["n"] == 300 and res["correct"] == int((want == labels).sum())
    assert res["agreement_with_float"] == float((pred.argmax(1) == want).mean())
    assert np.asarray(res["confusion"]).sum() == 300


@pytest.mark.gpu
def test_gpu_cli(gpu, tmp_path, capsys):
    net, cfg, _ = appendix_b_net(0)
    np.savez(str(tmp_path / "net.npz"), **net)
    with open(tmp_path / "config.json", "w") as f:
        json.dump({"indiv": {"net": {"params": cfg}}}, f)
    _write_benchmark(str(tmp_path / "benchmark.npz"), 64, 22, 1125, 4, 9)
    rc = E.main(["--net", str(tmp_path / "net.npz"), "--config", str(tmp_path / "config.json"),
                 "--benchmark", str(tmp_path / "benchmark.npz")])
    assert rc == 0
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    samples, labels, _ = E.load_benchmark(str(tmp_path / "benchmark.npz"))
    ps = ParamSet.from_quantlab(net, cfg)
    want = np.argmax(oracle.COracle(ps).batch(G.quantize_input(samples, ste_quant(net, "quant1")), nthreads=8), 1)
    assert res["correct"] == int((want == labels).sum())

"""The batched entry point inside a captured HIP graph (torch.cuda.CUDAGraph, i.e. hipGraph
stream capture): a serving loop can replay quantise -> forward -> class without host launch
overhead.  Parameters are uploaded on the first call, so one eager call precedes the capture
(an upload is a synchronous copy, which a capture may not contain)."""
import numpy as np
import pytest

import oracle
from oracle import golden_np as G
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu


def test_graph_capture_and_replay(gpu):
    import torch

    ps = ParamSet.synthetic(seed=51)
    lib.params_load(ps)
    co = oracle.COracle(ps)
    B = 3000
    rng = np.random.default_rng(51)
    xs = [rng.integers(-128, 128, size=(B, 22, 1125)).astype(np.int8) for _ in range(3)]
    xin = torch.from_numpy(xs[0]).cuda()
    lib.forward_torch(lib.pack_trials_torch(xin))  # eager call: uploads the parameters
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            logits = lib.forward_torch(lib.pack_trials_torch(xin, stream=s), stream=s)
            cls = lib.argmax_torch(logits, stream=s)
    for x in xs:  # new inputs copied into the captured buffer, then replay
        xin.copy_(torch.from_numpy(x))
        g.replay()
        torch.cuda.synchronize()
        want = co.batch(pack_trials(x), nthreads=8)
        assert np.array_equal(logits.cpu().numpy(), want)
        assert np.array_equal(cls.cpu().numpy(), np.argmax(want, axis=1))


def test_graph_float_path(gpu):
    """float EEG -> quantiser -> forward, captured once and replayed."""
    import torch

    ps = ParamSet.synthetic(seed=52)
    lib.params_load(ps)
    rng = np.random.default_rng(52)
    x = rng.normal(scale=0.9, size=(500, 22, 1125)).astype(np.float32)
    xin = torch.from_numpy(x).cuda()
    lib.forward_torch(lib.quantize_input_torch(xin, 1.3))
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = lib.forward_torch(lib.quantize_input_torch(xin, 1.3, stream=s), stream=s)
    g.replay()
    torch.cuda.synchronize()
    want = oracle.COracle(ps).batch(G.quantize_input(x, 1.3), nthreads=8)
    assert np.array_equal(out.cpu().numpy(), want)


def test_graph_keeps_its_parameter_set(gpu):
    """A graph captured under one parameter set keeps replaying that set's kernel variant and
    weights after a load that switches both build flags (plain BN, balanced clipping) and every
    weight: each set has its own device copy, which no later load overwrites."""
    import torch

    ps_a = ParamSet.synthetic(seed=53)
    ps_b = ParamSet.synthetic(seed=54, reorder_bn=False, clip_balanced=True)
    rng = np.random.default_rng(53)
    x = pack_trials(rng.integers(-128, 128, size=(700, 22, 1125)))
    want_a = oracle.COracle(ps_a).batch(x, nthreads=8)
    want_b = oracle.COracle(ps_b).batch(x, nthreads=8)
    assert not np.array_equal(want_a, want_b)
    xin = torch.from_numpy(x).cuda()
    lib.params_load(ps_a)
    lib.forward_torch(xin)  # eager call: uploads set A
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out_a = lib.forward_torch(xin, stream=s)
    lib.params_load(ps_b)
    eager_b = lib.forward_torch(xin)  # uploads set B to its own copy
    torch.cuda.synchronize()
    assert np.array_equal(eager_b.cpu().numpy(), want_b)
    out_a.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out_a.cpu().numpy(), want_a)
    # reloading A reuses its copy; the graph and eager calls agree again
    lib.params_load(ps_a)
    assert np.array_equal(lib.forward_torch(xin).cpu().numpy(), want_a)

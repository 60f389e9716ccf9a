"""Input quantiser: reference gen_input_header.py:66-76 with
functional.py:308-334 (quantize_to_int).  CPU tests pin the NumPy restatement on hand-computed
cases; GPU tests compare the HIP pre-pass with it bit for bit and run the full float-input path
(quantise on the GPU, then the fused forward) against the oracle."""
import numpy as np
import pytest

from oracle import golden_np as G


def test_quantize_known_cases():
    s = np.float32(2.0)
    x = np.array([[[0.0, 1.0, -1.0, 2.0, -2.0, 3.0, -5.0, 0.0157, -0.0157, 1.999, 0.00787402]]], dtype=np.float32)
    q = G.quantize_to_int(x, s)
    # x/s*127 truncated toward zero, clipped to +-127 (num_levels 255 never yields -128)
    want = np.trunc(np.clip(x.astype(np.float64) / 2.0, -1, 1) * 127.0)
    assert q.tolist()[0][0][:9] == [0, 63, -63, 127, -127, 127, -127, 0, 0]
    assert np.array_equal(q, want.astype(np.int64))


def test_quantize_float32_rounding_matters():
    # a value whose float32 quotient rounds up to an exact integer step while the exact
    # quotient is just below it: the restatement follows float32 arithmetic, like NumPy on the
    # reference's float32 arrays
    s = np.float32(3.0)
    x = np.nextafter(np.float32(3.0 * 10 / 127), np.float32(0), dtype=np.float32)
    q32 = G.quantize_to_int(np.array([[[x]]], dtype=np.float32), s)
    q64 = G.quantize_to_int(np.array([[[x]]], dtype=np.float64), s)
    assert q32.shape == q64.shape == (1, 1, 1)
    assert abs(int(q32[0, 0, 0]) - int(q64[0, 0, 0])) <= 1


def test_quantize_input_layout():
    rng = np.random.default_rng(3)
    x = rng.normal(size=(3, 5, 7)).astype(np.float32)
    out = G.quantize_input(x, 1.5)
    assert out.shape == (3, 48) and out.dtype == np.int8
    q = G.quantize_to_int(x, 1.5)
    for b in range(3):
        for t in range(7):
            for c in range(5):
                assert out[b, t * 5 + c] == q[b, c, t]
        assert not out[b, 35:].any()


def _boundary_inputs(rng, B, C, T, s, dtype):
    x = rng.normal(scale=s * 0.6, size=(B, C, T))
    flat = x.reshape(-1)
    k = rng.integers(-127, 128, size=flat.size // 3)
    # exact quantisation steps and their float neighbours
    steps = (k / 127.0 * s).astype(dtype)
    flat[: k.size] = steps
    flat[k.size: 2 * k.size] = np.nextafter(steps, np.inf, dtype=dtype)
    flat[2 * k.size: 2 * k.size + 50] = s * 4          # clipped
    flat[2 * k.size + 50: 2 * k.size + 100] = -s * 4
    return x.astype(dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("C,T", [(22, 1125), (64, 1000), (5, 70)])
def test_gpu_quantize_bit_exact(gpu, dtype, C, T):
    import torch
    from mibminet import lib

    rng = np.random.default_rng(C * T)
    s = 1.37
    x = _boundary_inputs(rng, 9, C, T, s, dtype)
    want = G.quantize_input(x, s)
    got = lib.quantize_input_torch(torch.from_numpy(x).to("cuda:0"), s).cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_float_input_path_end_to_end(gpu):
    """float EEG -> GPU quantiser -> fused forward == oracle(quantize_input(x))."""
    import torch
    import oracle
    from mibminet import lib
    from mibminet.params import ParamSet

    ps = ParamSet.synthetic(seed=11)
    lib.params_load(ps)
    rng = np.random.default_rng(5)
    x = rng.normal(scale=0.8, size=(40, 22, 1125)).astype(np.float32)
    xq = lib.quantize_input_torch(torch.from_numpy(x).to("cuda:0"), 1.1)
    y = lib.forward_torch(xq).cpu().numpy()
    want = oracle.COracle(ps).batch(G.quantize_input(x, 1.1), nthreads=4)
    assert np.array_equal(y, want)


def test_pack_abi_checks():
    from mibminet import lib

    L = lib.load()
    assert L.net_pack_trials_i8(None, None, 0, 22, 1125, 0, None) == 0  # empty batch
    assert L.net_pack_trials_i8(None, None, 1, 22, 1125, 0, None) == lib.NET_ERR_INVALID
    buf = np.zeros(64, np.int8)
    assert L.net_pack_trials_i8(buf.ctypes.data, buf.ctypes.data, 1, 65, 10, 0, None) == lib.NET_ERR_INVALID
    assert L.net_pack_trials_i8(buf.ctypes.data, buf.ctypes.data, 2**31, 22, 1125, 0, None) == lib.NET_ERR_INVALID
    # int trial indices in the kernel (b + gridDim.y must not wrap): B <= INT32_MAX - 65,535
    assert L.net_pack_trials_i8(buf.ctypes.data, buf.ctypes.data, 2**31 - 65535, 22, 1125, 0, None) == lib.NET_ERR_INVALID
    # the output must be 16-byte aligned (the tiles leave as 16-byte stores), and one trial's input
    # must stay below 2 GiB (one buffer view)
    base = (buf.ctypes.data + 15) // 16 * 16
    assert L.net_pack_trials_i8(buf.ctypes.data, base + 4, 1, 2, 3, 0, None) == lib.NET_ERR_INVALID
    assert L.net_quantize_input_f64(buf.ctypes.data, base, 1, 64, 2**22, 1.0, 0, None) == lib.NET_ERR_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("C,T,B", [(22, 1125, 300), (64, 1000, 70), (5, 70, 33), (3, 1, 2)])
def test_gpu_pack_trials_i8(gpu, C, T, B):
    """int8 [B][C][T] -> the batched [T][C] layout on the GPU == pack_trials (NumPy)."""
    import torch
    from mibminet import lib
    from mibminet.params import pack_trials

    rng = np.random.default_rng(C + T + B)
    x = rng.integers(-128, 128, size=(B, C, T)).astype(np.int8)
    got = lib.pack_trials_torch(torch.from_numpy(x).to("cuda:0")).cpu().numpy()
    assert np.array_equal(got, pack_trials(x))


@pytest.mark.gpu
def test_gpu_int8_channel_major_end_to_end(gpu):
    """int8 [B][C][T] -> GPU pack -> fused forward == oracle."""
    import torch
    import oracle
    from mibminet import lib
    from mibminet.params import ParamSet, pack_trials

    ps = ParamSet.synthetic(seed=12)
    lib.params_load(ps)
    rng = np.random.default_rng(6)
    x = rng.integers(-128, 128, size=(257, 22, 1125)).astype(np.int8)
    y = lib.forward_torch(lib.pack_trials_torch(torch.from_numpy(x).to("cuda:0"))).cpu().numpy()
    assert np.array_equal(y, oracle.COracle(ps).batch(pack_trials(x), nthreads=4))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_gpu_quantize_past_grid_limit(gpu, dtype):
    """B = 300,000 in one call == the NumPy restatement, for every trial.  A workgroup walks 2
    (float) or 4 (int8) trials, so the grid wants 150,000 / 75,000 rows: past grid.y's 65,535
    cap, where workgroups walk further trials, for every element type."""
    import torch
    from mibminet import lib

    B, C, T, s = 300_000, 5, 70, 0.93
    rng = np.random.default_rng(100)
    x = rng.normal(scale=0.7, size=(B, C, T)).astype(dtype)
    got = lib.quantize_input_torch(torch.from_numpy(x).to("cuda:0"), s).cpu().numpy()
    assert np.array_equal(got, G.quantize_input(x, s))
    xi = rng.integers(-128, 128, size=(B, C, T)).astype(np.int8)
    from mibminet.params import pack_trials
    assert np.array_equal(lib.pack_trials_torch(torch.from_numpy(xi).to("cuda:0")).cpu().numpy(), pack_trials(xi))


@pytest.mark.gpu
def test_gpu_float_path_config_b_100k(gpu):
    """Config-B float trials, B = 100,000 in one quantiser call (device-generated input), then the
    forward: sampled trials (random and the last 64) equal oracle(quantize_input(x))."""
    import torch
    import oracle
    from mibminet import lib
    from mibminet.params import ParamSet

    B = 100_000
    ps = ParamSet.synthetic(seed=13)
    lib.params_load(ps)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn((B, 22, 1125), dtype=torch.float32, device="cuda", generator=g) * 0.8
    xq = lib.quantize_input_torch(x, 1.1)
    y = lib.forward_torch(xq).cpu().numpy()
    idx = np.concatenate([np.random.default_rng(2).choice(B - 64, 128, replace=False), np.arange(B - 64, B)])
    xs = x[torch.from_numpy(idx).cuda()].cpu().numpy()
    want_q = G.quantize_input(xs, 1.1)
    assert np.array_equal(xq[torch.from_numpy(idx).cuda()].cpu().numpy(), want_q)
    assert np.array_equal(y[idx], oracle.COracle(ps).batch(want_q, nthreads=8))

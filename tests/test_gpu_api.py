"""C-ABI argument checks that need a visible device: device indices past the device count, and the
multi-device entry point's error path (shards enqueued before the failing one have finished when
the error is returned)."""
import ctypes

import numpy as np
import pytest

import oracle
from mibminet import lib
from mibminet.params import ParamSet, pack_trials

pytestmark = pytest.mark.gpu


def test_device_index_past_count(gpu):
    import torch

    L = lib.load()
    n = torch.cuda.device_count()
    lib.params_load(ParamSet.synthetic(seed=61))
    x = torch.zeros((4, lib.trial_stride()), dtype=torch.int8, device=gpu)
    y = torch.zeros((4, 4), dtype=torch.int8, device=gpu)
    c = torch.zeros(4, dtype=torch.int32, device=gpu)
    f = torch.zeros((4, 22, 1125), dtype=torch.float32, device=gpu)
    for dev in (n, 63, -1):
        assert L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), 4, dev, None) == lib.NET_ERR_INVALID
        assert L.net_argmax_batch(y.data_ptr(), c.data_ptr(), 4, 4, dev, None) == lib.NET_ERR_INVALID
        assert L.net_quantize_input_f32(f.data_ptr(), x.data_ptr(), 4, 22, 1125, ctypes.c_float(1.0), dev,
                                        None) == lib.NET_ERR_INVALID
        assert L.net_set_device(dev) == lib.NET_ERR_INVALID
        out = (ctypes.c_int32 * 3)()
        assert L.net_launch_info(4, dev, out) == lib.NET_ERR_INVALID
    assert L.net_set_device(0) == lib.NET_OK


def test_multi_error_waits_for_enqueued_shards(gpu):
    """On an error, net_model_compute_batch_multi returns only after the shards enqueued before
    the failing one have finished.  Checked without any synchronising call: right after the call
    the stream shard 0 ran on must already be idle (stream query), which fails if the wait is
    removed (shard 0 is a full 65,536-trial launch, ~0.4 ms, far longer than the call's return)."""
    import torch

    L = lib.load()
    ps = ParamSet.synthetic(seed=62)
    lib.params_load(ps)
    B = 65536
    stride = lib.trial_stride()
    g = torch.Generator(device="cuda").manual_seed(62)
    xd = torch.randint(-128, 128, (B, stride), dtype=torch.int8, device=gpu, generator=g)
    xd[:, 22 * 1125:] = 0
    y0 = torch.zeros((B, 4), dtype=torch.int8, device=gpu)
    raw = torch.zeros(16 + 4 * 4, dtype=torch.int8, device=gpu)
    idx = np.random.default_rng(62).choice(B, 256, replace=False)
    want = oracle.COracle(ps).batch(xd[torch.from_numpy(idx).cuda()].cpu().numpy(), nthreads=8)
    side = torch.cuda.Stream(device=gpu)
    torch.cuda.synchronize()
    for mode in ("null", "side"):
        y0.zero_()
        torch.cuda.synchronize()
        dev = (ctypes.c_int * 2)(0, 0)
        xp = (ctypes.c_void_p * 2)(xd.data_ptr(), xd.data_ptr() + 1)  # shard 1 misaligned
        yp = (ctypes.c_void_p * 2)(y0.data_ptr(), raw.data_ptr())
        bs = (ctypes.c_size_t * 2)(B, 4)
        st = torch.cuda.default_stream(gpu) if mode == "null" else side
        sp = None if mode == "null" else (ctypes.c_void_p * 2)(side.cuda_stream, side.cuda_stream)
        assert L.net_model_compute_batch_multi(2, dev, xp, yp, bs, sp) == lib.NET_ERR_INVALID
        # no sync before this: shard 0's stream must be idle already
        assert st.query(), f"{mode}: shard 0 still running when the error was returned"
        torch.cuda.synchronize()
        # shard 0, enqueued before the failing shard, ran to completion
        assert np.array_equal(y0.cpu().numpy()[idx], want)
    assert stride % 16 == 0


def test_param_images_bounded_and_reloadable(gpu):
    """12 distinct parameter sets in turn (more than the 8 device copies kept): every launch uses
    its own set, an evicted set reloads correctly, and unload + load works."""
    import torch

    rng = np.random.default_rng(70)
    x = pack_trials(rng.integers(-128, 128, size=(8, 22, 1125)))
    xd = torch.from_numpy(x).cuda()
    sets = [ParamSet.synthetic(seed=700 + i) for i in range(12)]
    for ps in sets + sets[:2]:
        lib.params_load(ps)
        assert np.array_equal(lib.forward_torch(xd).cpu().numpy(), oracle.COracle(ps).batch(x, nthreads=4))
    lib.params_unload()
    lib.params_load(sets[5])
    assert np.array_equal(lib.forward_torch(xd).cpu().numpy(), oracle.COracle(sets[5]).batch(x, nthreads=4))


def _upload_stats():
    L = lib.load()
    f = L.mibminet_test_upload_stats
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    a, b = ctypes.c_int64(), ctypes.c_int64()
    assert f(ctypes.byref(a), ctypes.byref(b)) == 0
    return a.value, b.value


def test_multi_first_call_uploads_before_enqueue(gpu):
    """A first multi-device call with a fresh parameter set uploads the image before the first
    shard is enqueued: no upload (a synchronous copy) happens between enqueues."""
    import torch

    L = lib.load()
    ps = ParamSet.synthetic(seed=64)
    lib.params_load(ps)
    x = pack_trials(np.random.default_rng(64).integers(-128, 128, size=(64, 22, 1125)))
    xd = torch.from_numpy(x).cuda()
    y = torch.zeros((64, 4), dtype=torch.int8, device=gpu)
    up0, upe0 = _upload_stats()
    n = 4
    dev = (ctypes.c_int * n)(*([0] * n))
    xp = (ctypes.c_void_p * n)(*[xd.data_ptr() + 16 * i * xd.shape[1] for i in range(n)])
    yp = (ctypes.c_void_p * n)(*[y.data_ptr() + 16 * 4 * i for i in range(n)])
    bs = (ctypes.c_size_t * n)(*([16] * n))
    assert L.net_model_compute_batch_multi(n, dev, xp, yp, bs, None) == 0
    up1, upe1 = _upload_stats()
    assert up1 == up0 + 1 and upe1 == upe0
    assert np.array_equal(y.cpu().numpy(), oracle.COracle(ps).batch(x, nthreads=4))


def test_param_copy_of_captured_graph_survives_reloads(gpu):
    """A launch captured into a HIP graph keeps its parameter copy however many other sets are
    loaded afterwards (the copy is never freed before net_params_unload), while copies that no
    launch can still read are evicted without a device synchronisation."""
    import torch

    L = lib.load()
    L.mibminet_test_device_images.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(71)
    x = pack_trials(rng.integers(-128, 128, size=(300, 22, 1125)))
    xd = torch.from_numpy(x).cuda()
    sets = [ParamSet.synthetic(seed=710 + i) for i in range(12)]
    lib.params_load(sets[0])
    lib.forward_torch(xd)  # uploads set 0 outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            out = lib.forward_torch(xd, stream=s)
    for ps in sets[1:]:  # 11 more sets: past the 8 copies kept per device
        lib.params_load(ps)
        assert np.array_equal(lib.forward_torch(xd).cpu().numpy(), oracle.COracle(ps).batch(x, nthreads=4))
    assert L.mibminet_test_device_images(0) <= 8
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.COracle(sets[0]).batch(x, nthreads=4))

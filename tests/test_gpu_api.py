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
    import torch

    L = lib.load()
    ps = ParamSet.synthetic(seed=62)
    lib.params_load(ps)
    rng = np.random.default_rng(62)
    x = pack_trials(rng.integers(-128, 128, size=(3000, 22, 1125)))
    want = oracle.COracle(ps).batch(x, nthreads=8)
    stride = lib.trial_stride()
    xd = torch.from_numpy(x).cuda()
    y0 = torch.zeros((3000, 4), dtype=torch.int8, device=gpu)
    raw = torch.zeros(16 + 4 * 4, dtype=torch.int8, device=gpu)
    for streams in (None, [torch.cuda.current_stream().cuda_stream] * 2):
        y0.zero_()
        dev = (ctypes.c_int * 2)(0, 0)
        xp = (ctypes.c_void_p * 2)(xd.data_ptr(), xd.data_ptr() + 1)  # shard 1 misaligned
        yp = (ctypes.c_void_p * 2)(y0.data_ptr(), raw.data_ptr())
        bs = (ctypes.c_size_t * 2)(3000, 4)
        sp = None if streams is None else (ctypes.c_void_p * 2)(*streams)
        assert L.net_model_compute_batch_multi(2, dev, xp, yp, bs, sp) == lib.NET_ERR_INVALID
        # shard 0, enqueued before the failing shard, ran to completion
        assert np.array_equal(y0.cpu().numpy(), want)
        assert stride % 16 == 0

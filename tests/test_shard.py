"""Static batch split: shard bounds, and a world_size-2 gloo run on CPU whose
per-rank shards (computed by the oracle in place of the GPU) concatenate to the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mibminet.params import ParamSet, pack_trials
from mibminet.shard import shard_bounds


@pytest.mark.parametrize("batch,world", [(0, 2), (1, 2), (7, 2), (65536, 8), (524288, 8), (13, 5)])
def test_shard_bounds_partition(batch, world):
    spans = [shard_bounds(batch, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == batch
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_shard_bounds_rejects():
    with pytest.raises(ValueError):
        shard_bounds(10, 0, 0)
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, blob, x, out_dir):
    import sys

    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import oracle
    from mibminet.params import ParamSet
    from mibminet.shard import forward_shard, gather_logits

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ps = ParamSet.from_blob(blob)
    co = oracle.COracle(ps)
    y = forward_shard(x, rank, world, compute=lambda part: co.batch(part, nthreads=1))
    full = gather_logits(y, x.shape[0], world)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("batch", [9, 16])
def test_gloo_world2_static_split(tmp_path, batch):
    import oracle

    ps = ParamSet.synthetic(seed=5, C=8, T=512)
    rng = np.random.default_rng(batch)
    x = pack_trials(rng.integers(-60, 60, size=(batch, 8, 512)))
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), ps.to_blob(), x, str(tmp_path)), nprocs=world, join=True)
    want = oracle.COracle(ps).batch(x, nthreads=2)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert np.array_equal(got, want)


def test_multi_abi_checks():
    from mibminet import lib

    L = lib.load()
    assert L.net_model_compute_batch_multi(0, None, None, None, None, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_multi(1, None, None, None, None, None) == lib.NET_ERR_INVALID
    assert L.net_model_compute_batch_multi(99, None, None, None, None, None) == lib.NET_ERR_INVALID


def test_forward_devices_rejects_wrong_layout():
    """A time-major batch passed as channel-major (or the reverse) is refused before any device
    work: the C ABI sees only pointers and counts and would return wrong logits."""
    from mibminet import lib
    from mibminet.shard import forward_devices

    lib.params_load(ParamSet.synthetic(seed=3))
    stride = lib.trial_stride()
    with pytest.raises(ValueError):
        forward_devices(np.zeros((4, stride), np.int8), [0], channel_major=True)
    with pytest.raises(ValueError):
        forward_devices(np.zeros((4, 22, 1125), np.int8), [0], channel_major=False)
    with pytest.raises(ValueError):
        lib.check_trial_shape((4, 22, 1000), True)
    lib.check_trial_shape((4, 22, 1125), True)
    lib.check_trial_shape((4, stride), False)


@pytest.mark.gpu
@pytest.mark.parametrize("devices,B", [([0], 1000), ([0, 0], 1001), ([0, 0, 0], 515)])
def test_gpu_forward_devices(gpu, devices, B):
    """One host thread, several shards (the same device listed several times stands in for the
    8-GPU node here): the concatenated logits equal the oracle's for the whole batch."""
    import oracle
    from mibminet import lib
    from mibminet.params import ParamSet, pack_trials
    from mibminet.shard import forward_devices

    ps = ParamSet.synthetic(seed=61)
    lib.params_load(ps)
    rng = np.random.default_rng(B)
    x = pack_trials(rng.integers(-128, 128, size=(B, 22, 1125)))
    assert np.array_equal(forward_devices(x, devices), oracle.COracle(ps).batch(x, nthreads=8))


def test_check_trials_contiguity_flag():
    """check_trials refuses strided batches at the raw-pointer entries; forward_devices copies
    every shard contiguously itself and accepts a strided view (dtype and shape still checked)."""
    from mibminet import lib

    lib.params_load(ParamSet.synthetic(seed=3))
    x = np.zeros((8, 22, 1125), np.int8)[::2]
    with pytest.raises(ValueError):
        lib.check_trials(x, True)
    lib.check_trials(x, True, require_contiguous=False)
    with pytest.raises(ValueError):
        lib.check_trials(x.astype(np.int16), True, require_contiguous=False)


@pytest.mark.gpu
def test_gpu_forward_devices_strided_view(gpu):
    """A strided view (every other trial of a larger batch) through forward_devices equals the
    oracle on the same trials."""
    import oracle
    from mibminet import lib
    from mibminet.shard import forward_devices

    ps = ParamSet.synthetic(seed=62)
    lib.params_load(ps)
    rng = np.random.default_rng(5)
    x = rng.integers(-128, 128, size=(300, 22, 1125)).astype(np.int8)
    view = x[::3]
    want = oracle.COracle(ps).batch(pack_trials(np.ascontiguousarray(view)), nthreads=8)
    assert np.array_equal(forward_devices(view, [0, 0], channel_major=True), want)

"""Static batch split of trials across GPUs (BASELINE config E).

Trials are independent (the reference's net_model_compute, edge-eegnet_wolf/src/cl/net/model.c:42,
has no cross-trial state), so a global batch is cut into contiguous per-rank shards, each rank
runs the fused forward on its own GPU, and the only exchange is the host-side concatenation of
the [B][N] logits after the fact.  There is no collective on the data path.

One process per GPU (torch.distributed.run): ``shard_bounds`` picks the rank's slice,
``forward_shard`` runs it through the C ABI on the rank's device, ``gather_logits`` collects the
shards on every rank (used by tests and tools, never inside a timed region).

One process for all GPUs (one host thread driving every device):
``forward_devices`` splits the batch the same way and runs all shards with one
``net_model_compute_batch_multi`` call.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_bounds(batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split [lo, hi) of ``batch`` trials for ``rank`` of ``world``; the first
    ``batch % world`` ranks take one extra trial."""
    if world < 1 or not 0 <= rank < world or batch < 0:
        raise ValueError(f"bad shard request batch={batch} world={world} rank={rank}")
    q, r = divmod(batch, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def forward_shard(x_global, rank: int, world: int, device: Optional[int] = None,
                  compute: Optional[Callable] = None):
    """Logits of this rank's shard of ``x_global`` ([B][trial_stride] int8).

    With ``compute`` None the shard is moved to ``device`` and run through
    ``net_model_compute_batch`` (lib.forward_torch); a ``compute`` callable (host arrays in,
    host arrays out) lets CPU-only tests exercise the split logic without a GPU."""
    lo, hi = shard_bounds(x_global.shape[0], world, rank)
    part = x_global[lo:hi]
    if compute is not None:
        return compute(part)
    import torch
    from . import lib

    dev = torch.device("cuda", device if device is not None else rank)
    xt = part.to(dev) if isinstance(part, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(part)).to(dev)
    return lib.forward_torch(xt).cpu().numpy()


def gather_logits(y_shard: np.ndarray, batch: int, world: int, n_out: int = 4) -> np.ndarray:
    """All-gather of the per-rank logits over the default process group (gloo or nccl): pads
    every shard to the largest shard size, gathers, trims, and returns the [batch][n_out]
    array on every rank."""
    import torch
    import torch.distributed as dist

    width = shard_bounds(batch, world, 0)[1]
    pad = np.zeros((width, n_out), dtype=np.int8)
    pad[: y_shard.shape[0]] = y_shard
    t = torch.from_numpy(pad.astype(np.int32))
    if dist.get_backend() == "nccl":
        t = t.cuda()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(batch, world, r)
        parts.append(outs[r].cpu().numpy()[: hi - lo].astype(np.int8))
    return np.concatenate(parts, axis=0)


def forward_devices(x_global, devices, channel_major: bool = False):
    """Logits of the whole batch ``x_global`` ([B][trial_stride] int8, or [B][C][T] with
    ``channel_major``; host array or tensor) split over ``devices`` with ``shard_bounds``: each
    shard is copied to its device, every device runs concurrently from this one host thread
    (net_model_compute_batch_multi / _multi_ct), and the [B][N] logits come back concatenated in
    trial order."""
    import torch
    from . import lib

    world = len(devices)
    # dtype and shape before any device work; each shard is copied contiguously below, so strided
    # views are fine here (model_compute_batch_multi checks the contiguous copies)
    lib.check_trials(x_global, channel_major, require_contiguous=False)
    xs, ys = [], []
    n_out = lib._dims().N
    for r, d in enumerate(devices):
        lo, hi = shard_bounds(x_global.shape[0], world, r)
        part = x_global[lo:hi]
        dev = torch.device("cuda", d)
        xt = part.to(dev) if isinstance(part, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(part)).to(dev)
        xs.append(xt.contiguous())
        ys.append(torch.empty((hi - lo, n_out), dtype=torch.int8, device=dev))
    for d in set(devices):
        torch.cuda.synchronize(d)  # the copies above ran on torch's streams
    lib.model_compute_batch_multi(xs, ys, list(devices), channel_major=channel_major)
    return np.concatenate([y.cpu().numpy() for y in ys], axis=0)

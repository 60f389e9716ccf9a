"""Accuracy harness: the step after the path.

The reference exports its evaluation set with ``QuantLab/export_net_data.py:89-105`` as
``benchmark.npz``: ``samples`` (float32 EEG trials, [n][1][1][C][T]), ``labels`` ([n]) and
``predictions`` (the float model's outputs, [n][1][N]).  QuantLab scores a network as the share
of trials whose ``torch.max(output, dim=1)`` index equals the label
(``quantlab/BCI-CompIV-2a/edgeEEGNet/postprocess.py:6-8``, ``utils/meter.py:36-39``).

This module runs that on the int8 path, all on the GPU: the input quantiser
(``net_quantize_input_f32``, quant1's absMaxValue), the fused forward
(``net_model_compute_batch_async``) and the class per trial (``net_argmax_batch``, first maximal
index on ties).  It reports the accuracy against the labels and the agreement with the float
model's own predictions.  No data set ships with the reference (``data/*.npz`` are gitignored),
so the tests drive it with synthetic files of the same layout.

    python -m mibminet.evaluate --net export/net.npz --config config.json --benchmark export/benchmark.npz
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import sys
from typing import Dict, Optional, Tuple

import numpy as np

from . import lib
from .params import ParamSet, ste_quant


def load_benchmark(path: str) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """Reads ``benchmark.npz`` (export_net_data.py:101): returns samples [n][C][T] float32, labels
    [n] int64 and the float predictions [n][N] (None when the file has none).  Loaded without
    pickle (``allow_pickle=False``)."""
    with np.load(path, allow_pickle=False) as f:
        s = np.asarray(f["samples"], dtype=np.float32)
        labels = np.asarray(f["labels"]).astype(np.int64).reshape(-1)
        pred = np.asarray(f["predictions"], dtype=np.float32) if "predictions" in f.files else None
    if s.ndim < 2:
        raise ValueError(f"samples must be [n][...][C][T], got shape {s.shape}")
    n = s.shape[0]
    samples = s.reshape(n, s.shape[-2], s.shape[-1])
    if labels.shape[0] != n:
        raise ValueError(f"{labels.shape[0]} labels for {n} samples")
    if pred is not None:
        pred = pred.reshape(n, -1)
    return np.ascontiguousarray(samples), labels, pred


def classify(ps: ParamSet, samples, scale: float, device: str = "cuda:0", batch: int = 65536):
    """Class per trial on the GPU.  ``samples``: float32 [n][C][T] (NumPy or a torch tensor);
    returns (classes int32 [n], logits int8 [n][N]) as device tensors."""
    import torch

    lib.params_load(ps)
    d = ps.dims
    x = torch.as_tensor(samples, dtype=torch.float32).to(device).contiguous()
    if x.dim() != 3 or x.shape[1] != d.C or x.shape[2] != d.T:
        raise ValueError(f"samples must be [n][{d.C}][{d.T}], got {tuple(x.shape)}")
    n = x.shape[0]
    logits = torch.empty((n, d.N), dtype=torch.int8, device=device)
    for lo in range(0, n, batch):
        hi = min(n, lo + batch)
        xq = lib.quantize_input_torch(x[lo:hi], float(scale))
        logits[lo:hi] = lib.forward_torch(xq)
    return lib.argmax_torch(logits), logits


def evaluate(ps: ParamSet, samples, labels, scale: float, predictions=None, device: str = "cuda:0",
             batch: int = 65536) -> Dict[str, object]:
    """Accuracy of the int8 path on a labelled set (and agreement with the float predictions)."""
    cls, _ = classify(ps, samples, scale, device, batch)
    got = cls.cpu().numpy().astype(np.int64)
    labels = np.asarray(labels, dtype=np.int64).reshape(-1)
    N = ps.dims.N
    conf = np.zeros((N, N), np.int64)  # [label][prediction]
    ok = (labels >= 0) & (labels < N)
    np.add.at(conf, (labels[ok], got[ok]), 1)
    out: Dict[str, object] = {
        "n": int(got.shape[0]),
        "correct": int((got == labels).sum()),
        "accuracy": float((got == labels).mean()) if got.size else 0.0,
        "confusion": conf.tolist(),
    }
    if predictions is not None:
        fp = np.asarray(predictions).reshape(got.shape[0], -1).argmax(axis=1)
        out["float_accuracy"] = float((fp == labels).mean()) if got.size else 0.0
        out["agreement_with_float"] = float((fp == got).mean()) if got.size else 0.0
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--net", required=True, help="QuantLab export net.npz (export_net_data.py:83-84)")
    ap.add_argument("--config", required=True, help="the experiment's config.json")
    ap.add_argument("--benchmark", required=True, help="benchmark.npz (export_net_data.py:89-101)")
    ap.add_argument("--plain-bn", action="store_true", help="the build without -DREORDER_BN")
    ap.add_argument("--clip-balanced", action="store_true", help="golden-model clip_balanced=True")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args(argv)
    with np.load(a.net, allow_pickle=False) as f:
        net = {k: f[k] for k in f.files}
    with open(a.config) as f:
        cfg = json.load(f)
    ps = ParamSet.from_quantlab(net, cfg["indiv"]["net"]["params"])
    ps = dataclasses.replace(ps, reorder_bn=not a.plain_bn, clip_balanced=a.clip_balanced)
    samples, labels, pred = load_benchmark(a.benchmark)
    res = evaluate(ps, samples, labels, ste_quant(net, "quant1"), pred, a.device)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""TEST INFRASTRUCTURE ONLY — NumPy restatement of the reference golden model.

Restates ``edge-eegnet_wolf/python_utils/golden_model.py`` (``GoldenModel(clip_balanced=...,
reorder_bn=...)`` with both flags taken from the ParamSet, Layer1..Layer5 at :153-379) and the functional ops it uses
(``python_utils/functional.py``), vectorised over a batch of trials.  It is independent of the C
restatement (oracle.c): the two are cross-checked on every fixture, and both are pinned by
SURVEY.md Appendix B's known answer.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Parameters come from ``mibminet.params.ParamSet`` (net.h arrays); the golden model holds the
same integers in torch order (``convert.inq_conv2d`` flips, ``np.convolve`` flips back), so the
views used here are ``ParamSet.w1()`` (L1, torch order), ``l2_weight_reverse`` (L2, torch order),
``w3_torch()`` (L3) and ``w5_flat()`` (L5).
"""
from __future__ import annotations

import numpy as np


def apply_factor_offset(x: np.ndarray, factor, offset=None, lo: int = -128) -> np.ndarray:
    """functional.py:55-91: trunc((x + offset) / factor), clip to [lo, 127] (lo = -128:
    clip_balanced=False; -127: clip_balanced=True, :89-91).

    ``x`` is [..., K, L] with the factor per K (second to last axis) or a scalar factor.
    Truncation toward zero is done with exact integer arithmetic (the reference divides in
    float64, which is exact for |x| < 2**53)."""
    x = np.asarray(x, dtype=np.int64)
    factor = np.asarray(factor, dtype=np.int64)
    if offset is None:
        offset = np.zeros_like(factor)
    offset = np.asarray(offset, dtype=np.int64)
    if factor.ndim == 1:
        factor = factor[:, None]
        offset = offset[:, None]
    num = x + offset
    q = np.abs(num) // np.abs(factor)
    q = np.where((num < 0) != (factor < 0), -q, q)
    return np.clip(q, lo, 127)


def relu(x: np.ndarray, threshold: np.ndarray) -> np.ndarray:
    """functional.py:94-115: max(x, threshold[k]) per channel k (axis -2)."""
    return np.maximum(x, np.asarray(threshold, dtype=np.int64)[:, None])


def pool(x: np.ndarray, n: int) -> np.ndarray:
    """functional.py:118-153 with shape (1, n), reduction "sum": floor(L/n) outputs, tail dropped."""
    L = x.shape[-1] // n
    return x[..., : L * n].reshape(*x.shape[:-1], L, n).sum(-1)


def xcorr_same(x: np.ndarray, w: np.ndarray, pad_start: int, pad_end: int) -> np.ndarray:
    """conv_time / depthwise_conv_time (functional.py:180-235): zero padding (K/2-1, K/2) and
    ``np.convolve(x, w_flipped, "valid")`` == cross-correlation with the torch-order filter.

    x: [B, K, L], w: [K, taps] (torch order) -> [B, K, L]."""
    taps = w.shape[-1]
    xp = np.pad(x, ((0, 0), (0, 0), (pad_start, pad_end)))
    win = np.lib.stride_tricks.sliding_window_view(xp, taps, axis=-1)  # [B, K, L, taps]
    return np.einsum("bklj,kj->bkl", win, np.asarray(w, np.int64), optimize=True)


def _lo(p) -> int:
    """GoldenModel(clip_balanced=...) (golden_model.py:43): the ParamSet's clip mode."""
    return -127 if getattr(p, "clip_balanced", False) else -128


def layer1(p, x: np.ndarray) -> np.ndarray:
    """Layer1.__call__ (golden_model.py:192-196): depthwise_conv_space + apply_factor_offset.
    x: [B, C, T] -> [B, F2, T]."""
    y = np.einsum("bct,fc->bft", x.astype(np.int64), p.w1().astype(np.int64), optimize=True)
    return apply_factor_offset(y, p.l1_factor, p.l1_offset, _lo(p))


def layer2(p, y1: np.ndarray) -> np.ndarray:
    """Layer2.__call__ reorder_bn=True (golden_model.py:241-247): conv_time, relu(-(bias//8)),
    sum-pool 8, apply_factor_offset.  [B, F2, T] -> [B, F2, T//8]."""
    a = xcorr_same(y1, p.l2_weight_reverse, 31, 32)
    if not getattr(p, "reorder_bn", True):
        # reorder_bn=False (golden_model.py:248-251): BN per element with factor//8, bias//8
        # (clip), relu at 0, sum-pool 8, // 8
        y = apply_factor_offset(a, p.l2_factor.astype(np.int64) // 8, p.l2_offset.astype(np.int64) // 8,
                                _lo(p))
        return pool(np.maximum(y, 0), 8) // 8
    thr = -(p.l2_offset.astype(np.int64) // 8)
    return apply_factor_offset(pool(relu(a, thr), 8), p.l2_factor, p.l2_offset, _lo(p))


def layer3(p, y2: np.ndarray) -> np.ndarray:
    """Layer3.__call__ (golden_model.py:285-289): depthwise_conv_time (pad 7/8), factor only."""
    a = xcorr_same(y2, p.w3_torch(), 7, 8)
    return apply_factor_offset(a, np.int64(p.l3_factor), lo=_lo(p))


def layer4(p, y3: np.ndarray) -> np.ndarray:
    """Layer4.__call__ reorder_bn=True (golden_model.py:330-337): pointwise_conv, relu, pool 8,
    apply_factor_offset.  [B, F2, T8] -> [B, F2, T64]."""
    b = np.einsum("bft,kf->bkt", y3.astype(np.int64), p.l4_weight.astype(np.int64), optimize=True)
    if not getattr(p, "reorder_bn", True):
        # reorder_bn=False (golden_model.py:337-340).  NB: the golden model clips each element to
        # int8 before the ReLU, the reference C (layer4.c:113-118) does not; the two only differ
        # when an element exceeds 127 (tests/test_variants.py pins both behaviours).
        y = apply_factor_offset(b, p.l4_factor.astype(np.int64) // 8, p.l4_offset.astype(np.int64) // 8,
                                _lo(p))
        return pool(np.maximum(y, 0), 8) // 8
    thr = -(p.l4_offset.astype(np.int64) // 8)
    return apply_factor_offset(pool(relu(b, thr), 8), p.l4_factor, p.l4_offset, _lo(p))


def layer5(p, y4: np.ndarray) -> np.ndarray:
    """Layer5.__call__ (golden_model.py:374-379): ravel, linear (+int bias), factor only."""
    B = y4.shape[0]
    z = y4.reshape(B, -1).astype(np.int64) @ p.w5_flat().astype(np.int64).T + p.l5_bias.astype(np.int64)
    q = np.abs(z) // abs(p.l5_factor)
    q = np.where((z < 0) != (p.l5_factor < 0), -q, q)
    return np.clip(q, _lo(p), 127)


def forward(p, x: np.ndarray, return_all: bool = False):
    """GoldenModel.__call__ (golden_model.py:104-107).  x: [B, C, T] or [C, T] int."""
    single = np.asarray(x).ndim == 2
    x = np.asarray(x, dtype=np.int64)
    if single:
        x = x[None]
    y1 = layer1(p, x)
    y2 = layer2(p, y1)
    y3 = layer3(p, y2)
    y4 = layer4(p, y3)
    z = layer5(p, y4)
    if single:
        y1, y2, y3, y4, z = y1[0], y2[0], y3[0], y4[0], z[0]
    if return_all:
        return z, (y1, y2, y3, y4)
    return z


def quantize_to_int(x: np.ndarray, scale_factor, num_levels: int = 255) -> np.ndarray:
    """functional.py:308-334 (quantize_to_int) in the input's own precision: x / scale, clip to
    [-1, 1], * (num_levels - 1) / 2 (evaluated left to right like the reference), truncated toward
    zero.  ``scale_factor`` is taken in x's dtype (the reference's absMaxValue is a float32
    scalar from net.npz, which NumPy keeps in float32 against a float32 array)."""
    assert num_levels % 2
    x = np.asarray(x)
    s = x.dtype.type(scale_factor)
    y = x / s
    y = np.clip(y, x.dtype.type(-1), x.dtype.type(1))
    y = y * x.dtype.type(num_levels - 1) / x.dtype.type(2)
    return np.trunc(y).astype(np.int64)


def quantize_input(x: np.ndarray, scale_factor) -> np.ndarray:
    """gen_input_header.py:66-76: quantize_to_int then transpose [B][C][T] -> [B][T][C], packed
    into the batched layout of the GPU path (trial stride = C*T rounded up to 16, pad zero)."""
    q = quantize_to_int(x, scale_factor)
    B, C, T = q.shape
    stride = (C * T + 15) // 16 * 16
    out = np.zeros((B, stride), dtype=np.int8)
    out[:, : C * T] = np.transpose(q, (0, 2, 1)).reshape(B, C * T).astype(np.int8)
    return out

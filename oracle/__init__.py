"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the MI-BMInet int8 forward pass.

``oracle.c`` restates the reference C layers (edge-eegnet_wolf/src/cl/net/layer{1..5}.c), and
``golden_np`` restates the reference NumPy golden model (python_utils/golden_model.py).
Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may import this package;
the product library never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

from . import golden_np  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")


class _Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("C", "T", "F1", "F2", "N", "C_ALIGN", "T_ALIGN", "T8", "T8_ALIGN", "T64", "T64_ALIGN")] + [
        ("l1_factor", ctypes.c_void_p), ("l1_offset", ctypes.c_void_p), ("l1_weight_align", ctypes.c_void_p),
        ("l2_factor", ctypes.c_void_p), ("l2_offset", ctypes.c_void_p), ("l2_weight_reverse", ctypes.c_void_p),
        ("l3_factor", ctypes.c_int32), ("l3_weight", ctypes.c_void_p),
        ("l4_factor", ctypes.c_void_p), ("l4_offset", ctypes.c_void_p), ("l4_weight", ctypes.c_void_p),
        ("l5_factor", ctypes.c_int32), ("l5_bias", ctypes.c_void_p), ("l5_weight", ctypes.c_void_p),
        ("reorder_bn", ctypes.c_int32), ("clip_lo", ctypes.c_int32),
    ]


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "oracle.c"))):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        for name in ("or_layer1", "or_layer2", "or_layer3", "or_layer4", "or_layer5", "or_model_compute"):
            getattr(_lib, name).argtypes = [vp, vp, vp]
            getattr(_lib, name).restype = None
        _lib.or_layer3_flip_inplace.argtypes = [vp, vp]
        _lib.or_model_compute_batch.argtypes = [vp, vp, sz, vp, sz, i]
    return _lib


class COracle:
    """ctypes view of oracle.c bound to one ParamSet (keeps the arrays alive)."""

    def __init__(self, ps):
        self.ps = ps
        d = ps.dims
        self._keep = [ps.l1_factor, ps.l1_offset, ps.l1_weight_align, ps.l2_factor, ps.l2_offset,
                      ps.l2_weight_reverse, ps.l3_weight, ps.l4_factor, ps.l4_offset, ps.l4_weight,
                      ps.l5_bias, ps.l5_weight]
        ptr = lambda a: a.ctypes.data
        self.p = _Params(d.C, d.T, d.F1, d.F2, d.N, d.C_ALIGN, d.T_ALIGN, d.T8, d.T8_ALIGN, d.T64, d.T64_ALIGN,
                         ptr(ps.l1_factor), ptr(ps.l1_offset), ptr(ps.l1_weight_align),
                         ptr(ps.l2_factor), ptr(ps.l2_offset), ptr(ps.l2_weight_reverse),
                         ps.l3_factor, ptr(ps.l3_weight),
                         ptr(ps.l4_factor), ptr(ps.l4_offset), ptr(ps.l4_weight),
                         ps.l5_factor, ptr(ps.l5_bias), ptr(ps.l5_weight), int(getattr(ps, "reorder_bn", True)),
                         -127 if getattr(ps, "clip_balanced", False) else -128)
        self.pref = ctypes.byref(self.p)
        self.L = lib()

    # reference-layout single-trial API
    def layer1(self, x_tc_align: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.ascontiguousarray(x_tc_align, np.int8).reshape(d.T, d.C_ALIGN)
        y = np.empty((d.F1, d.T_ALIGN), np.int8)
        self.L.or_layer1(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def layer2(self, y1: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.ascontiguousarray(y1, np.int8).reshape(d.F1, d.T_ALIGN)
        y = np.empty((d.F2, d.T8_ALIGN), np.int8)
        self.L.or_layer2(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def layer3(self, y2: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.ascontiguousarray(y2, np.int8).reshape(d.F2, d.T8_ALIGN)
        y = np.empty((d.F2, d.T8_ALIGN), np.int8)
        self.L.or_layer3(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def layer3_flip(self, y3: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        y = np.ascontiguousarray(y3, np.int8).reshape(d.F2, d.T8_ALIGN).copy()
        self.L.or_layer3_flip_inplace(self.pref, y.ctypes.data)
        return y

    def layer4(self, y3t: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.zeros(d.F2 * d.T8_ALIGN, np.int8)
        src = np.ascontiguousarray(y3t, np.int8).ravel()
        x[: src.size] = src[: x.size]
        y = np.empty((d.F2, d.T64_ALIGN), np.int8)
        self.L.or_layer4(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def layer5(self, y4: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.ascontiguousarray(y4, np.int8).reshape(d.F2, d.T64_ALIGN)
        y = np.empty(d.N, np.int8)
        self.L.or_layer5(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def model(self, x_tc_align: np.ndarray) -> np.ndarray:
        d = self.ps.dims
        x = np.ascontiguousarray(x_tc_align, np.int8).reshape(d.T, d.C_ALIGN)
        y = np.empty(d.N, np.int8)
        self.L.or_model_compute(self.pref, x.ctypes.data, y.ctypes.data)
        return y

    def batch(self, x_packed: np.ndarray, nthreads: int = 1) -> np.ndarray:
        """x_packed: [B][trial_stride] int8 (mibminet.params.pack_trials layout)."""
        x = np.ascontiguousarray(x_packed, np.int8)
        B = x.shape[0]
        y = np.empty((B, self.ps.dims.N), np.int8)
        self.L.or_model_compute_batch(self.pref, x.ctypes.data, x.shape[1], y.ctypes.data, B, nthreads)
        return y


def to_tc_align(x_ct: np.ndarray, C_ALIGN: int) -> np.ndarray:
    """[C][T] -> the reference single-trial layout [T][C_ALIGN] (gen_input_header.py:74-75)."""
    C, T = x_ct.shape
    out = np.zeros((T, C_ALIGN), np.int8)
    out[:, :C] = np.asarray(x_ct).T
    return out

"""ctypes binding of libmibminet.so (include/mibminet.h) — the Python mirror of the reference's
C model/layer API (edge-eegnet_wolf/src/cl/net/model.h, layers.h).

There is no CPU fallback: if the library cannot be loaded, or a call fails, a ``NetError`` is
raised.  Single-trial functions take host NumPy arrays in the reference layouts; the batched
function takes device pointers (e.g. ``torch.Tensor.data_ptr()`` of CUDA/HIP tensors).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from .params import ParamSet

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmibminet.so")

NET_OK = 0
NET_ERR_INVALID = -1
NET_ERR_NO_PARAMS = -2
NET_ERR_UNSUPPORTED = -3
NET_ERR_BLOB = -4
NET_ERR_RANGE = -5
NET_ERR_HIP = -100

EXPORTED_SYMBOLS = (
    "net_model_compute", "net_forward", "net_layer1", "net_layer2", "net_layer3",
    "net_layer3_flip_inplace", "net_layer4", "net_layer5", "net_last_error", "net_params_load",
    "net_params_dims", "net_params_unload", "net_trial_stride", "net_model_compute_batch",
    "net_model_compute_batch_async", "net_set_device", "net_launch_info", "net_error_string",
    "net_version", "net_quantize_input_f32", "net_quantize_input_f64", "net_argmax_batch",
    "net_pack_trials_i8", "net_model_compute_batch_multi", "net_model_compute_batch_ct",
    "net_model_compute_batch_multi_ct", "net_launch_info_ct", "net_model_compute_batch_f32",
    "net_model_compute_batch_ct_sync", "net_params_info", "net_params_load_arrays",
)
NET_PATH_FLOAT, NET_PATH_EXACT, NET_PATH_GENERAL = 0, 1, 2


class NetError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _lib_error_string(code)
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")


_lib: Optional[ctypes.CDLL] = None


def _lib_error_string(code: int) -> str:
    try:
        return load().net_error_string(code).decode()
    except Exception:  # pragma: no cover - library missing
        return "error"


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libmibminet.so (raises OSError — loudly — if it is missing or fails to load)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"libmibminet.so not found at {path}: build it with `make -C mi-bminet_amd`"
                      " (there is no CPU fallback)")
    L = ctypes.CDLL(path)
    vp, sz, i, i8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p
    for name in ("net_model_compute", "net_layer1", "net_layer2", "net_layer3", "net_layer4", "net_layer5"):
        getattr(L, name).argtypes = [i8p, i8p]
        getattr(L, name).restype = None
    L.net_forward.argtypes = [i8p, i8p]
    L.net_forward.restype = i
    L.net_layer3_flip_inplace.argtypes = [i8p]
    L.net_layer3_flip_inplace.restype = None
    L.net_last_error.argtypes = []
    L.net_last_error.restype = i
    L.net_params_load.argtypes = [vp, sz]
    L.net_params_load.restype = i
    L.net_params_dims.argtypes = [vp]
    L.net_params_dims.restype = i
    L.net_params_unload.argtypes = []
    L.net_params_unload.restype = None
    L.net_trial_stride.argtypes = []
    L.net_trial_stride.restype = sz
    L.net_model_compute_batch.argtypes = [vp, vp, sz, i]
    L.net_model_compute_batch.restype = i
    L.net_model_compute_batch_async.argtypes = [vp, vp, sz, i, vp]
    L.net_model_compute_batch_async.restype = i
    L.net_set_device.argtypes = [i]
    L.net_set_device.restype = i
    L.net_launch_info.argtypes = [sz, i, vp]
    L.net_launch_info.restype = i
    L.net_launch_info_ct.argtypes = [sz, i, vp]
    L.net_launch_info_ct.restype = i
    L.net_model_compute_batch_f32.argtypes = [vp, vp, sz, ctypes.c_float, i, vp]
    L.net_model_compute_batch_f32.restype = i
    L.net_error_string.argtypes = [i]
    L.net_error_string.restype = ctypes.c_char_p
    L.net_version.argtypes = []
    L.net_version.restype = i
    L.net_quantize_input_f32.argtypes = [vp, vp, sz, i, i, ctypes.c_float, i, vp]
    L.net_quantize_input_f32.restype = i
    L.net_quantize_input_f64.argtypes = [vp, vp, sz, i, i, ctypes.c_double, i, vp]
    L.net_quantize_input_f64.restype = i
    L.net_model_compute_batch_multi.argtypes = [i, vp, vp, vp, vp, vp]
    L.net_model_compute_batch_multi.restype = i
    L.net_pack_trials_i8.argtypes = [vp, vp, sz, i, i, i, vp]
    L.net_pack_trials_i8.restype = i
    L.net_argmax_batch.argtypes = [vp, vp, sz, i, i, vp]
    L.net_argmax_batch.restype = i
    L.net_model_compute_batch_ct.argtypes = [vp, vp, sz, i, vp]
    L.net_model_compute_batch_ct.restype = i
    L.net_model_compute_batch_multi_ct.argtypes = [i, vp, vp, vp, vp, vp]
    L.net_model_compute_batch_multi_ct.restype = i
    L.net_model_compute_batch_ct_sync.argtypes = [vp, vp, sz, i]
    L.net_model_compute_batch_ct_sync.restype = i
    L.net_params_info.argtypes = [vp]
    L.net_params_info.restype = i
    # test hooks (include/mibminet_testing.h)
    L.mibminet_test_force_general.argtypes = [i]
    L.mibminet_test_folded_filters.argtypes = [vp]
    L.mibminet_test_folded_filters.restype = i
    L.mibminet_test_force_general.restype = i
    L.mibminet_test_xdiv_host.argtypes = [vp, sz, ctypes.c_int32, vp]
    L.mibminet_test_xdiv_host.restype = i
    L.mibminet_test_xdiv_gpu.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, vp, i]
    L.mibminet_test_xdiv_gpu.restype = i
    L.mibminet_test_pool_consts.argtypes = [ctypes.c_int32, ctypes.c_int32, vp, vp]
    L.mibminet_test_pool_consts.restype = i
    L.mibminet_test_params_xr.argtypes = []
    L.mibminet_test_params_xr.restype = i
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != NET_OK:
        raise NetError(rc, what)


# ---- parameters -------------------------------------------------------------------------------
_loaded: Optional[ParamSet] = None


def params_load(ps: ParamSet) -> None:
    """net_params_load(blob) — replaces the generated net.h globals of the reference."""
    global _loaded
    blob = ps.to_blob()
    buf = ctypes.create_string_buffer(blob, len(blob))
    _check(load().net_params_load(buf, len(blob)), "net_params_load")
    _loaded = ps


def params_load_blob(blob: bytes) -> None:
    global _loaded
    buf = ctypes.create_string_buffer(blob, len(blob))
    _check(load().net_params_load(buf, len(blob)), "net_params_load")
    _loaded = ParamSet.from_blob(blob)


def params_dims() -> dict:
    arr = (ctypes.c_int32 * 7)()
    rc = load().net_params_dims(arr)
    if rc == NET_ERR_NO_PARAMS:
        return {}
    _check(rc, "net_params_dims")
    return dict(zip(("C", "T", "F1", "F2", "N", "weight_bits", "loaded"), list(arr)))


def params_unload() -> None:
    global _loaded
    load().net_params_unload()
    _loaded = None


def trial_stride() -> int:
    return int(load().net_trial_stride())


def _dims():
    if _loaded is None:
        raise NetError(NET_ERR_NO_PARAMS, "no parameters loaded")
    return _loaded.dims


# ---- reference single-trial API (host arrays, reference layouts) --------------------------------
def _call_void(name: str, x: np.ndarray, out: np.ndarray) -> np.ndarray:
    L = load()
    getattr(L, name)(x.ctypes.data, out.ctypes.data)
    _check(L.net_last_error(), name)
    return out


def net_model_compute(x_tc_align: np.ndarray) -> np.ndarray:
    """model.h:40 — x: [T][C_ALIGN] int8 -> logits [N] int8."""
    d = _dims()
    x = np.ascontiguousarray(x_tc_align, np.int8).reshape(d.T, d.C_ALIGN)
    return _call_void("net_model_compute", x, np.empty(d.N, np.int8))


def net_layer1(x_tc_align: np.ndarray) -> np.ndarray:
    d = _dims()
    x = np.ascontiguousarray(x_tc_align, np.int8).reshape(d.T, d.C_ALIGN)
    return _call_void("net_layer1", x, np.empty((d.F1, d.T_ALIGN), np.int8))


def net_layer2(y1: np.ndarray) -> np.ndarray:
    d = _dims()
    x = np.ascontiguousarray(y1, np.int8).reshape(d.F1, d.T_ALIGN)
    return _call_void("net_layer2", x, np.empty((d.F2, d.T8_ALIGN), np.int8))


def net_layer3(y2: np.ndarray) -> np.ndarray:
    d = _dims()
    x = np.ascontiguousarray(y2, np.int8).reshape(d.F2, d.T8_ALIGN)
    return _call_void("net_layer3", x, np.empty((d.F2, d.T8_ALIGN), np.int8))


def net_layer3_flip_inplace(y3: np.ndarray) -> np.ndarray:
    """layers.h:107 — [F2][T8_ALIGN] -> [T8][F2] (in place on a copy; returned)."""
    d = _dims()
    buf = np.ascontiguousarray(y3, np.int8).reshape(d.F2 * d.T8_ALIGN).copy()
    L = load()
    L.net_layer3_flip_inplace(buf.ctypes.data)
    _check(L.net_last_error(), "net_layer3_flip_inplace")
    return buf


def net_layer4(y3t: np.ndarray) -> np.ndarray:
    d = _dims()
    x = np.zeros(d.F2 * d.T8_ALIGN, np.int8)
    src = np.ascontiguousarray(y3t, np.int8).ravel()
    x[: min(src.size, x.size)] = src[: x.size]
    return _call_void("net_layer4", x, np.empty((d.F2, d.T64_ALIGN), np.int8))


def net_layer5(y4: np.ndarray) -> np.ndarray:
    d = _dims()
    x = np.ascontiguousarray(y4, np.int8).reshape(d.F2, d.T64_ALIGN)
    return _call_void("net_layer5", x, np.empty(d.N, np.int8))


def set_device(device: int) -> None:
    _check(load().net_set_device(device), "net_set_device")


# ---- batched device API -----------------------------------------------------------------------
def model_compute_batch(x_ptr: int, y_ptr: int, B: int, device: int = 0, stream: Optional[int] = None) -> None:
    """net_model_compute_batch(_async): x_ptr/y_ptr are device pointers ([B][trial_stride] int8
    and [B][N] int8).  With ``stream`` the launch is enqueued without a host sync."""
    L = load()
    if stream is None:
        _check(L.net_model_compute_batch(x_ptr, y_ptr, B, device), "net_model_compute_batch")
    else:
        _check(L.net_model_compute_batch_async(x_ptr, y_ptr, B, device, stream), "net_model_compute_batch_async")


def model_compute_batch_ct_sync(x_ptr: int, y_ptr: int, B: int, device: int = 0) -> None:
    """net_model_compute_batch_ct_sync (SURVEY §8(b)'s signature): channel-major [B][C][T] int8
    trials and [B][N] logits, device pointers; waits for completion."""
    _check(load().net_model_compute_batch_ct_sync(x_ptr, y_ptr, B, device), "net_model_compute_batch_ct_sync")


def params_info() -> dict:
    """net_params_info: which kernels the loaded set runs ("float", "exact" or "general"), and for
    "exact" the first layer / filter whose requant has no proven float form."""
    arr = (ctypes.c_int32 * 5)()
    _check(load().net_params_info(arr), "net_params_info")
    path = {NET_PATH_FLOAT: "float", NET_PATH_EXACT: "exact", NET_PATH_GENERAL: "general"}[arr[0]]
    return {"path": path, "layer": arr[1], "filter": arr[2], "shape": arr[3], "exact_division": bool(arr[4])}


def force_general(on: bool) -> None:
    """Test hook (mibminet_test_force_general): later loads run the run-time-dimension kernels
    even for the compiled geometries."""
    _check(load().mibminet_test_force_general(1 if on else 0), "mibminet_test_force_general")


def folded_filters() -> int:
    """Test hook (mibminet_test_folded_filters): constant filters the loaded set had folded."""
    v = ctypes.c_int32(0)
    _check(load().mibminet_test_folded_filters(ctypes.byref(v)), "mibminet_test_folded_filters")
    return v.value


def params_exact_division() -> bool:
    """True when the loaded set runs the exact integer-division kernels (Cfg::XR: a set outside the
    float requant envelope), False for the float-requant kernels."""
    rc = load().mibminet_test_params_xr()
    if rc < 0:
        raise NetError(rc, "mibminet_test_params_xr")
    return bool(rc)


def xdiv_host(e: np.ndarray, d: int) -> np.ndarray:
    """The exact-division kernels' integer division emulated on the host (mibminet_test_xdiv_host)."""
    e = np.ascontiguousarray(e, dtype=np.int32)
    q = np.empty_like(e)
    _check(load().mibminet_test_xdiv_host(e.ctypes.data, e.size, int(d), q.ctypes.data), "mibminet_test_xdiv_host")
    return q


def xdiv_gpu_mismatches(d: int, e0: int, count: int, device: int = 0) -> int:
    """The device xdiv over e0 .. e0 + count - 1 against C division (mibminet_test_xdiv_gpu)."""
    n = ctypes.c_int64(0)
    _check(load().mibminet_test_xdiv_gpu(int(d), int(e0), int(count), ctypes.byref(n), device), "mibminet_test_xdiv_gpu")
    return int(n.value)


def launch_info(B: int, device: int = 0, channel_major: bool = False) -> dict:
    arr = (ctypes.c_int32 * 3)()
    fn = load().net_launch_info_ct if channel_major else load().net_launch_info
    _check(fn(B, device, arr), "net_launch_info")
    return {"grid": arr[0], "threads": arr[1], "lds_bytes": arr[2]}


def forward_torch(x, params: Optional[ParamSet] = None, stream=None):
    """Convenience: x is a CUDA/HIP int8 torch tensor [B][trial_stride] -> logits [B][N] tensor."""
    import torch

    if params is not None:
        params_load(params)
    d = _dims()
    if x.dtype != torch.int8 or not x.is_cuda or not x.is_contiguous():
        raise ValueError("x must be a contiguous int8 device tensor [B][trial_stride]")
    B = x.shape[0]
    if x.numel() != B * trial_stride():
        raise ValueError(f"x must be [B][{trial_stride()}]")
    y = torch.empty((B, d.N), dtype=torch.int8, device=x.device)
    s = torch.cuda.current_stream(x.device) if stream is None else stream
    model_compute_batch(x.data_ptr(), y.data_ptr(), B, x.device.index or 0, s.cuda_stream)
    return y


def forward_ct_torch(x, stream=None):
    """net_model_compute_batch_ct: x is a CUDA/HIP int8 tensor [B][C][T] (channel-major, the
    reference's input.npz layout; any byte alignment) -> logits [B][N] tensor, with no separate
    transpose pass."""
    import torch

    d = _dims()
    if x.dtype != torch.int8 or not x.is_cuda or not x.is_contiguous() or tuple(x.shape[1:]) != (d.C, d.T):
        raise ValueError(f"x must be a contiguous int8 device tensor [B][{d.C}][{d.T}]")
    B = x.shape[0]
    y = torch.empty((B, d.N), dtype=torch.int8, device=x.device)
    s = torch.cuda.current_stream(x.device) if stream is None else stream
    _check(load().net_model_compute_batch_ct(x.data_ptr(), y.data_ptr(), B, x.device.index or 0, s.cuda_stream),
           "net_model_compute_batch_ct")
    return y


def forward_f32_torch(x, scale: float, stream=None):
    """net_model_compute_batch_f32: x is a CUDA/HIP float32 tensor [B][C][T] (float EEG, the
    reference's input.npz layout) -> logits [B][N], quantised inside the fused kernel."""
    import torch

    d = _dims()
    if x.dtype != torch.float32 or not x.is_cuda or not x.is_contiguous() or tuple(x.shape[1:]) != (d.C, d.T):
        raise ValueError(f"x must be a contiguous float32 device tensor [B][{d.C}][{d.T}]")
    B = x.shape[0]
    y = torch.empty((B, d.N), dtype=torch.int8, device=x.device)
    s = torch.cuda.current_stream(x.device) if stream is None else stream
    _check(load().net_model_compute_batch_f32(x.data_ptr(), y.data_ptr(), B, scale, x.device.index or 0,
                                              s.cuda_stream), "net_model_compute_batch_f32")
    return y


def quantize_input_torch(x, scale: float, stream=None):
    """Input quantiser (net_quantize_input_f32/_f64): x is a CUDA/HIP float32 or float64 tensor
    [B][C][T] (the reference's input.npz layout); returns the batched int8 layout [B][stride]
    (stride = C*T rounded up to 16, each trial [T][C]) that forward_torch consumes.  Semantics of
    the reference's quantize_to_int (functional.py:308-334) in the input's precision."""
    import torch

    if not x.is_cuda or not x.is_contiguous() or x.dim() != 3 or x.dtype not in (torch.float32, torch.float64):
        raise ValueError("x must be a contiguous float32/float64 device tensor [B][C][T]")
    B, C, T = x.shape
    stride = (C * T + 15) // 16 * 16
    y = torch.empty((B, stride), dtype=torch.int8, device=x.device)
    s = torch.cuda.current_stream(x.device) if stream is None else stream
    fn = load().net_quantize_input_f32 if x.dtype == torch.float32 else load().net_quantize_input_f64
    _check(fn(x.data_ptr(), y.data_ptr(), B, C, T, scale, x.device.index or 0, s.cuda_stream), "net_quantize_input")
    return y


def argmax_torch(logits, stream=None):
    """Class per trial (net_argmax_batch): logits is a CUDA/HIP int8 tensor [B][N]; returns an int32
    tensor [B] holding the first maximal index of each row (torch.max(dim=1)'s rule)."""
    import torch

    if logits.dtype != torch.int8 or not logits.is_cuda or not logits.is_contiguous() or logits.dim() != 2:
        raise ValueError("logits must be a contiguous int8 device tensor [B][N]")
    B, N = logits.shape
    out = torch.empty((B,), dtype=torch.int32, device=logits.device)
    s = torch.cuda.current_stream(logits.device) if stream is None else stream
    _check(load().net_argmax_batch(logits.data_ptr(), out.data_ptr(), B, N, logits.device.index or 0, s.cuda_stream),
           "net_argmax_batch")
    return out


def pack_trials_torch(x, stream=None):
    """net_pack_trials_i8: x is a CUDA/HIP int8 tensor [B][C][T] (channel-major); returns the
    batched layout [B][stride] (each trial [T][C], pad zero) that forward_torch consumes."""
    import torch

    if x.dtype != torch.int8 or not x.is_cuda or not x.is_contiguous() or x.dim() != 3:
        raise ValueError("x must be a contiguous int8 device tensor [B][C][T]")
    B, C, T = x.shape
    stride = (C * T + 15) // 16 * 16
    y = torch.empty((B, stride), dtype=torch.int8, device=x.device)
    s = torch.cuda.current_stream(x.device) if stream is None else stream
    _check(load().net_pack_trials_i8(x.data_ptr(), y.data_ptr(), B, C, T, x.device.index or 0, s.cuda_stream),
           "net_pack_trials_i8")
    return y


def check_trials(x, channel_major: bool, require_contiguous: bool = True) -> None:
    """Raises ValueError unless ``x`` (NumPy array or torch tensor) is a C-contiguous int8 batch of
    trials in the chosen layout (check_trial_shape).  The C ABI sees only pointers and counts, so a
    batch of another element type (e.g. int64 from rng.integers) or with strides would otherwise
    run and its bytes be read as int8 trials.  ``require_contiguous=False``: callers that copy the
    batch contiguously themselves before it reaches a pointer (shard.forward_devices)."""
    dt = str(getattr(x, "dtype", ""))
    if dt not in ("int8", "torch.int8"):
        raise ValueError(f"trials must be int8, got {dt or type(x).__name__}")
    contiguous = x.is_contiguous() if hasattr(x, "is_contiguous") else bool(x.flags["C_CONTIGUOUS"])
    if require_contiguous and not contiguous:
        raise ValueError("trials must be C-contiguous")
    check_trial_shape(tuple(x.shape), channel_major)


def check_trial_shape(shape, channel_major: bool) -> None:
    """Raises ValueError unless ``shape`` is a batch of trials in the chosen layout: [B][C][T]
    (channel-major) or [B][trial_stride] (time-major).  The C ABI sees only pointers and counts, so
    a batch in the other layout would otherwise run and return wrong logits."""
    d = _dims()
    want = (d.C, d.T) if channel_major else (trial_stride(),)
    if len(shape) != 1 + len(want) or tuple(shape[1:]) != want:
        kind = f"[B][{d.C}][{d.T}] (channel-major)" if channel_major else f"[B][{want[0]}] (time-major)"
        raise ValueError(f"trials must be {kind}, got {tuple(shape)}")


def model_compute_batch_multi(xs, ys, devices, channel_major: bool = False) -> None:
    """net_model_compute_batch_multi(_ct): xs[i] / ys[i] are device tensors on devices[i]
    ([B_i][trial_stride], or [B_i][C][T] with ``channel_major``, and [B_i][N] int8); one host call
    runs every shard and waits for all."""
    n = len(devices)
    if not (len(xs) == len(ys) == n):
        raise ValueError("xs, ys and devices must have the same length")
    d = _dims()
    for x, y in zip(xs, ys):
        check_trials(x, channel_major)
        if tuple(y.shape) != (x.shape[0], d.N):
            raise ValueError(f"logits must be [B][{d.N}] per shard, got {tuple(y.shape)}")
    dev = (ctypes.c_int * n)(*devices)
    xp = (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])
    yp = (ctypes.c_void_p * n)(*[y.data_ptr() for y in ys])
    bs = (ctypes.c_size_t * n)(*[x.shape[0] for x in xs])
    fn = load().net_model_compute_batch_multi_ct if channel_major else load().net_model_compute_batch_multi
    _check(fn(n, dev, xp, yp, bs, None), "net_model_compute_batch_multi")

"""The C-ABI library loads without a GPU, exports every symbol include/mibminet.h declares and
validates parameters on the host.  No compute calls are made here."""
import ctypes
import os
import re

import numpy as np
import pytest

from mibminet import lib
from mibminet.params import ParamSet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "mibminet.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(net_\w+)\s*\(", text, flags=re.M)))


def test_header_symbols_exported():
    L = lib.load()
    names = declared_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(lib.EXPORTED_SYMBOLS)


def test_section_8b_signature():
    """SURVEY §8(b)'s batched entry, int f(const int8_t* x /*[B][C][T]*/, int8_t* y /*[B][N]*/,
    size_t B, int device), exists with exactly those argument types (channel-major trials), and
    the time-major entry of the same shape tells a [B][C][T] caller where to go."""
    text = open(os.path.join(ROOT, "include", "mibminet.h")).read()
    decl = re.search(r"int\s+net_model_compute_batch_ct_sync\s*\(([^)]*)\)", text)
    assert decl, "net_model_compute_batch_ct_sync is not declared"
    args = [re.sub(r"\s+", " ", a.strip()) for a in decl.group(1).split(",")]
    assert args == ["const int8_t* x", "int8_t* y", "size_t B", "int device"]
    L = lib.load()
    fn = L.net_model_compute_batch_ct_sync
    assert [t.__name__ for t in fn.argtypes] == ["c_void_p", "c_void_p", "c_ulong", "c_int"]
    assert fn.restype is ctypes.c_int
    at = text.index("int net_model_compute_batch(")
    doc = text[text.rindex("/*", 0, at):at]
    assert "net_model_compute_batch_ct_sync" in doc and "[B][C][T]" in doc
    # no device work without parameters: the entry validates before touching the GPU
    lib.params_unload()
    assert fn(None, None, 0, 0) == lib.NET_ERR_NO_PARAMS


def test_version_and_errors():
    L = lib.load()
    assert L.net_version() == 1
    assert L.net_error_string(0) == b"ok"
    assert b"blob" in L.net_error_string(lib.NET_ERR_BLOB)


@pytest.mark.parametrize("C,T,wbits", [(22, 1125, 8), (64, 1000, 8), (22, 1125, 4)])
def test_params_load_host(C, T, wbits):
    ps = ParamSet.synthetic(seed=9, C=C, T=T, weight_bits=wbits)
    lib.params_load(ps)
    d = lib.params_dims()
    assert (d["C"], d["T"], d["F1"], d["F2"], d["N"], d["weight_bits"], d["loaded"]) == (C, T, 16, 16, 4, wbits, 1)
    assert lib.trial_stride() == (C * T + 15) // 16 * 16
    lib.params_unload()
    assert lib.params_dims() == {}
    assert lib.trial_stride() == 0


def test_params_load_rejects():
    L = lib.load()
    bad = b"x" * 100
    assert L.net_params_load(bad, len(bad)) == lib.NET_ERR_BLOB
    ps = ParamSet.synthetic(seed=1)
    blob = ps.to_blob()
    assert L.net_params_load(blob[:-4], len(blob) - 4) == lib.NET_ERR_BLOB
    # a geometry without a compiled kernel runs the general kernels (forward_gen.hpp)
    ps2 = ParamSet.synthetic(seed=1, C=8, T=512, N=3)
    b2 = ps2.to_blob()
    assert L.net_params_load(b2, len(b2)) == lib.NET_OK
    assert lib.params_info() == {"path": "general", "layer": 0, "filter": -1, "shape": -1, "exact_division": False}
    # outside every kernel (T > 4096, N > 16, F1 != 16) fails loudly
    for kw in (dict(C=8, T=4104), dict(C=8, T=512, N=17), dict(C=8, T=512, F1=8)):
        b = ParamSet.synthetic(seed=1, **kw).to_blob()
        assert L.net_params_load(b, len(b)) == lib.NET_ERR_UNSUPPORTED, kw
    ps1 = ParamSet.synthetic(seed=1)
    b1 = ps1.to_blob()
    assert L.net_params_load(b1, len(b1)) == lib.NET_OK
    assert lib.params_info() == {"path": "float", "layer": 0, "filter": -1, "shape": 0, "exact_division": False}
    # offsets beyond the float envelope load (exact-division kernels); past int32 they are refused
    ps3 = ParamSet.synthetic(seed=1)
    ps3.l1_offset[0] = 4_500_000
    b3 = ps3.to_blob()
    # ... onto the +127 rail with the calibrated factor: folded, float kernels
    assert L.net_params_load(b3, len(b3)) == lib.NET_OK and L.mibminet_test_params_xr() == 0
    assert lib.folded_filters() == 1
    ps3.l1_factor[0] = 1 << 16  # outputs that still vary: exact division
    b3 = ps3.to_blob()
    assert L.net_params_load(b3, len(b3)) == lib.NET_OK and L.mibminet_test_params_xr() == 1
    # the public query names the requant that forced the exact path
    assert lib.params_info() == {"path": "exact", "layer": 1, "filter": 0, "shape": 0, "exact_division": True}
    ps3.l1_offset[0] = 2 ** 31 - 1
    b3 = ps3.to_blob()
    assert L.net_params_load(b3, len(b3)) == lib.NET_ERR_RANGE


def test_no_params_errors():
    lib.params_unload()
    L = lib.load()
    x = np.zeros((1125, 24), np.int8)
    y = np.zeros(4, np.int8)
    assert L.net_forward(x.ctypes.data, y.ctypes.data) == lib.NET_ERR_NO_PARAMS
    L.net_model_compute(x.ctypes.data, y.ctypes.data)
    assert L.net_last_error() == lib.NET_ERR_NO_PARAMS
    assert L.net_model_compute_batch(None, None, 0, 0) == lib.NET_ERR_NO_PARAMS


def test_appendix_b_factors_accepted():
    """The real-looking (Appendix B) factors pass the exact-reciprocal verification."""
    from mibminet.params import appendix_b_net
    net, cfg, _ = appendix_b_net(0)
    lib.params_load(ParamSet.from_quantlab(net, cfg))
    lib.params_unload()


def test_params_load_rejects_nonzero_pads():
    """Pad weights the reference multiplies (func_dotp over C_ALIGN and F2 * T64_ALIGN bytes,
    layer1.c:90, layer5.c:81) must be zero, as ParamSet.validate requires: the C ABI rejects a blob
    whose pads are not (NET_ERR_BLOB), and accepts the unpatched blob."""
    L = lib.load()
    ps = ParamSet.synthetic(seed=3)
    blob = bytearray(ps.to_blob())
    assert L.net_params_load(bytes(blob), len(blob)) == lib.NET_OK
    # layer-1 weights follow the 64-byte header and the two int32[F2] arrays; row f has C_ALIGN bytes
    C, CA, F2 = ps.dims.C, ps.dims.C_ALIGN, 16
    assert CA > C
    b1 = bytearray(blob)
    b1[64 + 2 * 4 * F2 + 3 * CA + C] = 1  # filter 3, first pad channel
    assert L.net_params_load(bytes(b1), len(b1)) == lib.NET_ERR_BLOB
    # layer-5 weights end the blob: [N][F2][T64_ALIGN]; the last byte is a pad column (T64 = 17 < 20)
    assert ps.dims.T64 < ps.dims.T64_ALIGN
    b5 = bytearray(blob)
    b5[-1] = 0xFF
    assert L.net_params_load(bytes(b5), len(b5)) == lib.NET_ERR_BLOB
    lib.params_unload()


def _multi_order(devices, fail_at=-1):
    L = lib.load()
    f = L.mibminet_test_multi_order
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    dev = (ctypes.c_int * len(devices))(*devices)
    buf = ctypes.create_string_buffer(256)
    rc = f(len(devices), dev, fail_at, buf, 256)
    return rc, buf.value.decode().split()


def test_multi_driver_prepares_every_device_before_enqueueing():
    """net_model_compute_batch_multi's driver (run with recording stand-ins, no device): every
    listed device receives the parameter image (P, once per distinct device) before the first
    shard is enqueued (E), so the first call on a multi-GPU node uploads up front and then starts
    all devices back to back; then all shards are waited for (W)."""
    rc, log = _multi_order([0, 1, 2, 3, 4, 5, 6, 7])
    assert rc == 0
    assert log == [f"P{d}" for d in range(8)] + [f"E{i}" for i in range(8)] + ["W8"]
    rc, log = _multi_order([0, 1, 0, 1])
    assert log == ["P0", "P1", "E0", "E1", "E2", "E3", "W4"]


def test_multi_driver_error_waits_for_enqueued_shards_only():
    rc, log = _multi_order([0, 1, 2, 3], fail_at=2)
    assert rc == lib.NET_ERR_INVALID
    assert log == ["P0", "P1", "P2", "P3", "E0", "E1", "E2", "W2"]

"""The reference's generated weight sources (net.h / net.c, gen_net_header.py:49-224 in
header_file.py's format) load in C with no blob and no Python: net_params_load_arrays, with
include/mibminet_net_h.h filling its struct from the NET_* macros and net_l* globals.

CPU only: the writer (mibminet/net_h.py) round-trips every array through a compiled net.c, and the
device image built from the arrays is byte-identical to the one built from the blob.  The GPU run
of the linked C host is tests/test_c_host.py::test_c_host_linked_net_h."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from mibminet import lib
from mibminet.net_h import net_h_sources, write_net_h
from mibminet.params import ParamSet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "c_host")
sys.path.insert(0, EX)
import make_nets  # noqa: E402


def test_committed_nets_are_the_writers_output(tmp_path):
    make_nets.main(str(tmp_path))
    for name in make_nets.NETS:
        for f in ("net.h", "net.c"):
            assert (tmp_path / name / f).read_bytes() == open(os.path.join(EX, name, f), "rb").read(), (name, f)


def test_reference_format():
    """The generator's own layout: #include "rt/rt_api.h", #define dimensions, extern RT_L2_DATA
    const declarations in net.h, initialised arrays in net.c."""
    ps = ParamSet.synthetic(seed=1)
    h, c = net_h_sources(ps)
    assert h.startswith("#ifndef __NET_NET_H__\n#define __NET_NET_H__\n\n#include \"rt/rt_api.h\"\n")
    for line in ("#define NET_C 22\n", "#define NET_T8_ALIGN 140\n", "#define NET_T64_ALIGN 20\n",
                 "#define NET_N 4\n", f"#define NET_L3_FACTOR {ps.l3_factor}\n",
                 "extern RT_L2_DATA const int8_t net_l1_weight_align[384];\n",
                 "extern RT_L2_DATA const int8_t net_l5_weight[1280];\n",
                 "extern RT_L2_DATA const int32_t net_l2_offset[16];\n"):
        assert line in h, line
    assert c.startswith('#include "net.h"\n') and "RT_L2_DATA const int8_t net_l2_weight_reverse[] = {\n" in c
    assert max(len(l) for l in c.splitlines()) <= 102  # 100-column wrap, "};" after the last line
    with pytest.raises(ValueError):
        net_h_sources(ParamSet.synthetic(seed=1, weight_bits=4))


def _compile_net_c(tmp_path, ps):
    write_net_h(ps, str(tmp_path), runtime_include=None)
    so = tmp_path / "libnet.so"
    subprocess.run(["gcc", "-O1", "-fPIC", "-shared", "-std=c11", "-I", str(tmp_path), "-o", str(so),
                    str(tmp_path / "net.c")], check=True)
    return ctypes.CDLL(str(so))


def _arrays(L, ps, flags):
    d = ps.dims
    A = lib.load()
    A.net_params_load_arrays.argtypes = [ctypes.c_void_p]

    class Arrays(ctypes.Structure):
        _fields_ = [(n, ctypes.c_int32) for n in ("C", "T", "F1", "F2", "D", "N")] + [("flags", ctypes.c_uint32)] + [
            (n, ctypes.c_void_p) for n in ("l1_factor", "l1_offset", "l1_weight_align", "l2_factor", "l2_offset",
                                           "l2_weight_reverse")] + [("l3_factor", ctypes.c_int32),
                                                                    ("l3_weight", ctypes.c_void_p)] + [
            (n, ctypes.c_void_p) for n in ("l4_factor", "l4_offset", "l4_weight")] + [
            ("l5_factor", ctypes.c_int32), ("l5_bias", ctypes.c_void_p), ("l5_weight", ctypes.c_void_p)]

    sym = lambda n: ctypes.cast(getattr(L, n), ctypes.c_void_p).value  # noqa: E731
    return Arrays(d.C, d.T, d.F1, d.F2, d.D, d.N, flags,
                  sym("net_l1_factor"), sym("net_l1_offset"), sym("net_l1_weight_align"), sym("net_l2_factor"),
                  sym("net_l2_offset"), sym("net_l2_weight_reverse"), ps.l3_factor, sym("net_l3_weight"),
                  sym("net_l4_factor"), sym("net_l4_offset"), sym("net_l4_weight"), ps.l5_factor,
                  sym("net_l5_bias"), sym("net_l5_weight"))


def _digest():
    A = lib.load()
    A.mibminet_test_image_digest.argtypes = [ctypes.c_void_p]
    v = ctypes.c_uint64(0)
    assert A.mibminet_test_image_digest(ctypes.byref(v)) == lib.NET_OK
    return v.value


@pytest.mark.parametrize("kw", [dict(C=22, T=1125), dict(C=19, T=480, N=3), dict(C=64, T=1000, reorder_bn=False),
                                dict(C=38, T=960, N=2, clip_balanced=True, stress=True)])
def test_arrays_round_trip_and_load_like_the_blob(tmp_path, kw):
    ps = ParamSet.synthetic(seed=7, **kw)
    L = _compile_net_c(tmp_path, ps)
    # every array of the compiled net.c holds the ParamSet's values, in its layout
    for name, ctype, want in (("net_l1_factor", ctypes.c_int32, ps.l1_factor),
                              ("net_l1_weight_align", ctypes.c_int8, ps.l1_weight_align),
                              ("net_l2_weight_reverse", ctypes.c_int8, ps.l2_weight_reverse),
                              ("net_l2_weight", ctypes.c_int8, ps.l2_weight_reverse[:, ::-1]),
                              ("net_l3_weight", ctypes.c_int8, ps.l3_weight),
                              ("net_l4_offset", ctypes.c_int32, ps.l4_offset),
                              ("net_l5_bias", ctypes.c_int8, ps.l5_bias),
                              ("net_l5_weight", ctypes.c_int8, ps.l5_weight)):
        got = np.ctypeslib.as_array((ctype * want.size).in_dll(L, name))
        np.testing.assert_array_equal(got, np.asarray(want).ravel(), err_msg=name)
    # the arrays load through the C entry into the same device image as the blob
    lib.params_load(ps)
    want_digest = _digest()
    info = lib.params_info()
    a = _arrays(L, ps, ps.flags)
    lib.params_unload()
    assert lib.load().net_params_load_arrays(ctypes.byref(a)) == lib.NET_OK
    assert _digest() == want_digest and lib.params_info() == info
    # the blob's checks: non-zero pads and unknown flags are refused
    a.flags = 4
    assert lib.load().net_params_load_arrays(ctypes.byref(a)) == lib.NET_ERR_BLOB
    assert lib.load().net_params_load_arrays(None) == lib.NET_ERR_INVALID
    lib.params_unload()


def test_linked_hosts_build():
    subprocess.run(["make", "-s", "-C", EX], check=True)
    for b in ("net_host_b22", "net_host_g19"):
        r = subprocess.run([os.path.join(EX, b)], capture_output=True, text=True)
        assert r.returncode == 2 and "usage" in r.stderr

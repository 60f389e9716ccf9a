#!/usr/bin/env python3
"""Launch geometry (grid, threads, LDS) the library picks for the time-major and channel-major
kernels of config B (diagnostic): python tools/occ.py [lib.so ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet.params import ParamSet  # noqa: E402

blob = ParamSet.synthetic(seed=1).to_blob()
for p in sys.argv[1:] or [os.path.join(ROOT, "mi-bminet_amd", "mibminet", "libmibminet.so")]:
    L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
    L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    assert L.net_params_load(blob, len(blob)) == 0
    for name in ("net_launch_info", "net_launch_info_ct"):
        out = (ctypes.c_int32 * 3)()
        rc = getattr(L, name)(ctypes.c_size_t(65536), 0, out)
        print(f"{os.path.basename(p):24s} {name:20s} rc {rc} grid {out[0]} threads {out[1]} lds {out[2]}")

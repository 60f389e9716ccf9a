#!/usr/bin/env python3
"""Same-box A/B timing of library builds (diagnostic; not part of the product).

Loads each given libmibminet variant (tools/build_diag.sh builds them with -D flags), loads the
same synthetic parameter blob into each, and times net_model_compute_batch_async on one resident
batch, interleaving the variants round by round so clock drift hits all of them alike.

    python tools/ab.py [--cfg b22|c64] [--B 65536] [--iters 20] [--rounds 5] lib1.so lib2.so ...
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet.params import ParamSet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="b22")
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--settle", type=float, default=1.0, help="seconds of untimed launches before round 0")
    ap.add_argument("--variant", default="canonical", choices=("canonical", "plain_bn", "clip_balanced"))
    ap.add_argument("--ct", action="store_true", help="channel-major input (net_model_compute_batch_ct)")
    ap.add_argument("--f32", action="store_true", help="float32 channel-major input (net_model_compute_batch_f32)")
    ap.add_argument("--extreme", action="store_true", help="ParamSet.synthetic_extreme (the exact-division kernels)")
    ap.add_argument("--force-general", action="store_true",
                    help="run the compiled geometries on the general kernels (mibminet_test_force_general)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    C, T, N = {"b22": (22, 1125, 4), "c64": (64, 1000, 4), "p64": (64, 480, 4), "g19": (19, 1125, 3),
               "g38": (38, 480, 2), "g16": (16, 1125, 4), "g32": (32, 960, 2), "p64l": (64, 960, 4),
               "g64t": (64, 1125, 4), "g48l": (48, 2000, 3)}[a.cfg]
    mk = ParamSet.synthetic_extreme if a.extreme else ParamSet.synthetic
    blob = mk(1, C=C, T=T, N=N, reorder_bn=a.variant != "plain_bn",
              clip_balanced=a.variant == "clip_balanced").to_blob()
    libs = []
    for p in a.libs:
        L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
        L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.net_trial_stride.restype = ctypes.c_size_t
        L.net_model_compute_batch_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                    ctypes.c_int, ctypes.c_void_p]
        if a.ct:
            L.net_model_compute_batch_ct.argtypes = L.net_model_compute_batch_async.argtypes
            L.net_model_compute_batch_async = L.net_model_compute_batch_ct
        if a.f32:  # same call shape, the scale bound in (3 sigma of the standard-normal input)
            f = L.net_model_compute_batch_f32
            f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float, ctypes.c_int,
                          ctypes.c_void_p]
            L.net_model_compute_batch_async = (lambda f: lambda x, y, B, d, s: f(x, y, B, 3.0, d, s))(f)
        if a.force_general:
            L.mibminet_test_force_general(1)
        rc = L.net_params_load(blob, len(blob))
        assert rc == 0, (p, rc)
        libs.append(L)
    stride = C * T if a.ct else libs[0].net_trial_stride()
    if a.f32:
        x = torch.randn((a.B, C, T), dtype=torch.float32, device="cuda:0")
    else:
        x = torch.randint(-128, 128, (a.B, stride), dtype=torch.int8, device="cuda:0")
    y = torch.empty((a.B, N), dtype=torch.int8, device="cuda:0")
    st = torch.cuda.current_stream()
    outs = []
    for L in libs:
        y.zero_()
        assert L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), a.B, 0, st.cuda_stream) == 0
        outs.append(y.clone())
    for p, o in zip(a.libs, outs):
        same = bool(torch.equal(o, outs[0]))
        print(f"{os.path.basename(p):28s} output {'==' if same else '!='} first library's", flush=True)
    # settle the clock (power cap) before the first timed round: without it the first library of
    # the first rounds can read a few per cent slow (identical libraries differed by up to 3.7 %)
    import time
    t0 = time.time()
    while time.time() - t0 < a.settle:
        for L in libs:
            for _ in range(10):
                L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), a.B, 0, st.cuda_stream)
        torch.cuda.synchronize()
    times = {p: [] for p in a.libs}
    for r in range(a.rounds):
        for p, L in zip(a.libs, libs):
            for _ in range(2):
                L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), a.B, 0, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                rc = L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), a.B, 0, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            assert rc == 0, (p, rc)
            times[p].append(e0.elapsed_time(e1) / a.iters)
        print(f"round {r}: " + "  ".join(f"{os.path.basename(p)}={times[p][-1]:.4f}" for p in a.libs), flush=True)
    base = statistics.median(times[a.libs[0]])
    for p in a.libs:
        m = statistics.median(times[p])
        print(f"{os.path.basename(p):28s} median {m:.4f} ms  ({(m / base - 1) * 100:+.1f}% vs first)")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Kernel time against batch size (diagnostic; not part of the product): fits t(B) = t0 + B * c
over back-to-back launches, so the per-launch fixed cost (prologue, ramp, drain) shows as t0.

    python tools/bsweep.py [--cfg b22] [--iters 30] [--rounds 5] lib.so [B ...]
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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("lib")
    ap.add_argument("Bs", nargs="*", type=int, default=[512, 4096, 16384, 32768, 65536, 131072])
    a = ap.parse_args()
    C, T = {"b22": (22, 1125), "c64": (64, 1000)}[a.cfg]
    blob = ParamSet.synthetic(seed=1, C=C, T=T).to_blob()
    L = ctypes.CDLL(os.path.abspath(a.lib), mode=ctypes.RTLD_LOCAL)
    L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.net_trial_stride.restype = ctypes.c_size_t
    L.net_model_compute_batch_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_int, ctypes.c_void_p]
    assert L.net_params_load(blob, len(blob)) == 0
    stride = L.net_trial_stride()
    Bmax = max(a.Bs)
    x = torch.randint(-128, 128, (Bmax, stride), dtype=torch.int8, device="cuda:0")
    y = torch.empty((Bmax, 4), dtype=torch.int8, device="cuda:0")
    st = torch.cuda.current_stream()
    times = {B: [] for B in a.Bs}
    for _ in range(100):
        L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), 65536, 0, st.cuda_stream)
    for r in range(a.rounds):
        for B in a.Bs:
            for _ in range(3):
                L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), B, 0, st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), B, 0, st.cuda_stream)
            e1.record(st)
            e1.synchronize()
            times[B].append(e0.elapsed_time(e1) / a.iters)
    med = {B: statistics.median(v) for B, v in times.items()}
    for B in a.Bs:
        print(f"B={B:7d}  {med[B]:.4f} ms  {med[B] * 1e3 / B * 1e3:.3f} ns/trial", flush=True)
    Bs = sorted(a.Bs)
    if len(Bs) >= 2:
        b0, b1 = Bs[-2], Bs[-1]
        c = (med[b1] - med[b0]) / (b1 - b0)
        print(f"slope {c * 1e6:.3f} ns/trial; intercept at B={b1}: {med[b1] - c * b1:.4f} ms")


if __name__ == "__main__":
    main()

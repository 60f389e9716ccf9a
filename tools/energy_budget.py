#!/usr/bin/env python3
"""Energy per launch of the fused forward and of its ablation builds (diagnostic).

For each library (tools/build_diag.sh builds the MIB_DIAG_* ablations) it runs 65,536-trial
launches back to back for --seconds on one resident batch, samples rocm-smi board power and sclk
alongside (power_sample.sampler), and prints ms per launch, the median power, the median sclk and
the energy per launch (median power x time), plus the change of each against the first line.
"base:zero" runs the first library on an all-zero batch (no data toggling).

    python tools/energy_budget.py [--seconds 3] lib1.so [lib2.so ...]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from mibminet.params import ParamSet  # noqa: E402
from power_sample import sampler  # noqa: E402


def medians(samples):
    pw, ck = [], []
    for _, txt in samples:
        try:
            d = json.loads(txt)
            card = d[sorted(k for k in d if k.startswith("card"))[0]]
            for k, v in card.items():
                if "Power" in k and "W" in k:
                    pw.append(float(v))
                if k.startswith("sclk"):
                    ck.append(float(str(v).strip("()Mhz")))
        except Exception:
            pass
    med = lambda v: sorted(v)[len(v) // 2] if v else float("nan")  # noqa: E731
    return med(pw), med(ck), len(pw)


def run(L, x, y, B, seconds):
    st = torch.cuda.current_stream()
    for _ in range(50):
        L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), B, 0, st.cuda_stream)
    torch.cuda.synchronize()
    stop, samples = threading.Event(), []
    th = threading.Thread(target=sampler, args=(stop, samples))
    th.start()
    t0 = time.time()
    n = 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    while time.time() - t0 < seconds:
        for _ in range(100):
            L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), B, 0, st.cuda_stream)
        n += 100
        torch.cuda.synchronize()
    e1.record(st)
    e1.synchronize()
    stop.set()
    th.join()
    return e0.elapsed_time(e1) / n, samples


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    blob = ParamSet.synthetic(seed=1).to_blob()
    B = 65536
    rows = []
    xr = xz = None
    for i, p in enumerate(a.libs):
        L = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
        L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.net_trial_stride.restype = ctypes.c_size_t
        L.net_model_compute_batch_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                                    ctypes.c_void_p]
        assert L.net_params_load(blob, len(blob)) == 0
        if xr is None:
            stride = L.net_trial_stride()
            xr = torch.randint(-128, 128, (B, stride), dtype=torch.int8, device="cuda")
            xz = torch.zeros((B, stride), dtype=torch.int8, device="cuda")
            y = torch.empty((B, 4), dtype=torch.int8, device="cuda")
        for zero in ((False, True) if i == 0 else (False,)):
            ms, samples = run(L, xz if zero else xr, y, B, a.seconds)
            w, mhz, n = medians(samples)
            name = os.path.basename(p) + (":zero" if zero else "")
            rows.append((name, ms, w, mhz, ms * w / 1e3))
            print(f"{name:28s} {ms:.4f} ms/launch  {w:6.0f} W  {mhz:6.0f} MHz  {ms * w / 1e3:.4f} J/launch  "
                  f"({n} power samples)", flush=True)
    e0, t0 = rows[0][4], rows[0][1]
    print("# name, ms, W, sclk MHz, J/launch, time vs first, energy vs first")
    for name, ms, w, mhz, e in rows:
        print(f"{name:28s} {ms:.4f} {w:6.0f} {mhz:6.0f} {e:.4f} {(ms / t0 - 1) * 100:+6.1f}% {(e / e0 - 1) * 100:+6.1f}%")


if __name__ == "__main__":
    main()

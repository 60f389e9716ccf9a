#!/usr/bin/env python3
"""Sustained-load power/clock sample (diagnostic): runs the batched forward back to back for
--seconds on one resident batch and samples rocm-smi power and sclk while it runs.

    python tools/power_sample.py [--lib path] [--seconds 4] [--zero]
"""
import argparse
import ctypes
import os
import subprocess
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet.params import ParamSet  # noqa: E402


def sampler(stop, out):
    while not stop.is_set():
        try:
            r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True, text=True, timeout=5)
            out.append((time.time(), r.stdout))
        except Exception as e:  # pragma: no cover
            out.append((time.time(), str(e)))
        time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "mi-bminet_amd/mibminet/libmibminet.so"))
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--zero", action="store_true")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.abspath(a.lib), mode=ctypes.RTLD_LOCAL)
    L.net_params_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.net_trial_stride.restype = ctypes.c_size_t
    L.net_model_compute_batch_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    blob = ParamSet.synthetic(seed=1).to_blob()
    assert L.net_params_load(blob, len(blob)) == 0
    B = 65536
    stride = L.net_trial_stride()
    x = torch.zeros((B, stride), dtype=torch.int8, device="cuda") if a.zero else \
        torch.randint(-128, 128, (B, stride), dtype=torch.int8, device="cuda")
    y = torch.empty((B, 4), dtype=torch.int8, device="cuda")
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
    while time.time() - t0 < a.seconds:
        for _ in range(100):
            L.net_model_compute_batch_async(x.data_ptr(), y.data_ptr(), B, 0, st.cuda_stream)
        n += 100
        torch.cuda.synchronize()
    e1.record(st)
    e1.synchronize()
    stop.set()
    th.join()
    ms = e0.elapsed_time(e1) / n
    print(f"{os.path.basename(a.lib)} zero={a.zero}: {n} launches, {ms:.4f} ms/launch, {B / ms * 1e3:.4g} trials/s")
    import json
    pw, ck = [], []
    for t, txt in samples:
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
    if pw:
        print(f"  power W: n={len(pw)} median {sorted(pw)[len(pw) // 2]:.0f} max {max(pw):.0f}")
    if ck:
        print(f"  sclk MHz: n={len(ck)} median {sorted(ck)[len(ck) // 2]:.0f} min {min(ck):.0f}")
    if not pw and samples:
        print("  raw sample:", samples[len(samples) // 2][1][:800])


if __name__ == "__main__":
    main()

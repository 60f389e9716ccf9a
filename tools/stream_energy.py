#!/usr/bin/env python3
"""Time and board power of a plain HBM read stream over config B's input bytes (diagnostic).

Reads a 1.6223 GB uniform-random buffer (65,536 trials x 24,754 B, rounded to 16 B) with
tools/stream_probe.hip at several grid sizes, back to back for --seconds each, with rocm-smi
sampled alongside (power_sample.sampler).  Prints ms per pass, GB/s, W, sclk and J per pass: the
energy the memory system alone spends on the bytes the forward kernel must read.

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o tools/libstream_probe.so tools/stream_probe.hip
    python tools/stream_energy.py [--seconds 4]
"""
import argparse
import ctypes
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from energy_budget import medians  # noqa: E402
from power_sample import sampler  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--blocks", default="512,1024,2048")
    a = ap.parse_args()
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libstream_probe.so"))
    L.stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    nbytes = (65536 * (22 * 1125 + 4) + 15) // 16 * 16
    x = torch.randint(-128, 128, (nbytes,), dtype=torch.int8, device="cuda")
    out = torch.empty(4096 * 512, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    for blocks in (int(b) for b in a.blocks.split(",")):
        for _ in range(20):
            assert L.stream_read(x.data_ptr(), nbytes, out.data_ptr(), blocks, st.cuda_stream) == 0
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
                L.stream_read(x.data_ptr(), nbytes, out.data_ptr(), blocks, st.cuda_stream)
            n += 100
            torch.cuda.synchronize()
        e1.record(st)
        e1.synchronize()
        stop.set()
        th.join()
        ms = e0.elapsed_time(e1) / n
        w, mhz, ns = medians(samples)
        print(f"stream blocks={blocks:5d}: {ms:.4f} ms/pass  {nbytes / ms / 1e6:7.0f} GB/s  {w:6.0f} W  {mhz:6.0f} MHz  "
              f"{ms * w / 1e3:.4f} J/pass  ({ns} power samples)", flush=True)


if __name__ == "__main__":
    main()

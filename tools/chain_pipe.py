#!/usr/bin/env python3
"""Float EEG -> class per trial, serial against chunked and pipelined over two streams
(diagnostic).  The pipeline quantises chunk i + 1 (HBM-bound) while the fused forward runs chunk i
(power-bound), through a ring of int8 chunk buffers small enough to stay in the 256 MB Infinity
Cache between the two kernels.

    python tools/chain_pipe.py [--B 65536] [--chunks 2048,4096,8192,16384] [--reps 10]
"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet import lib  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--chunks", default="2048,4096,8192,16384")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--nbuf", type=int, default=2)
    ap.add_argument("--cfg", default="b22", choices=("b22", "c64", "p64"))
    a = ap.parse_args()
    C, T = {"b22": (22, 1125), "c64": (64, 1000), "p64": (64, 480)}[a.cfg]
    B = a.B
    lib.params_load(ParamSet.synthetic(seed=1, C=C, T=T))
    stride = lib.trial_stride()
    L = lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    xf = torch.randn((B, C, T), dtype=torch.float32, device=dev, generator=g) * 50.0
    scale = ctypes.c_float(200.0)
    cls = torch.empty((B,), dtype=torch.int32, device=dev)
    logits = torch.empty((B, 4), dtype=torch.int8, device=dev)
    ybig = torch.empty((B, stride), dtype=torch.int8, device=dev)
    s0 = torch.cuda.current_stream(dev)

    def serial():
        L.net_quantize_input_f32(xf.data_ptr(), ybig.data_ptr(), B, C, T, scale, 0, s0.cuda_stream)
        L.net_model_compute_batch_async(ybig.data_ptr(), logits.data_ptr(), B, 0, s0.cuda_stream)
        L.net_argmax_batch(logits.data_ptr(), cls.data_ptr(), B, 4, 0, s0.cuda_stream)

    def timed(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for _ in range(a.reps):
            fn()
        e1.record(s0)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    serial()
    torch.cuda.synchronize()
    want = cls.clone()
    print(f"serial: {timed(serial):.3f} ms per {B} trials", flush=True)

    def fused():  # the float entry: quantised inside the forward kernel
        L.net_model_compute_batch_f32(xf.data_ptr(), logits.data_ptr(), B, scale, 0, s0.cuda_stream)
        L.net_argmax_batch(logits.data_ptr(), cls.data_ptr(), B, 4, 0, s0.cuda_stream)

    cls.zero_()
    fused()
    torch.cuda.synchronize()
    print(f"fused float entry: {timed(fused):.3f} ms per {B} trials, same classes: {bool(torch.equal(cls, want))}",
          flush=True)
    sq, sf = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for K in [int(k) for k in a.chunks.split(",")]:
        bufs = [torch.empty((K, stride), dtype=torch.int8, device=dev) for _ in range(a.nbuf)]
        freed = [torch.cuda.Event() for _ in range(a.nbuf)]
        ready = [torch.cuda.Event() for _ in range(a.nbuf)]

        def pipe():
            done = torch.cuda.Event()
            sq.wait_stream(s0)
            sf.wait_stream(s0)
            n = (B + K - 1) // K
            for i in range(n):
                lo, hi = i * K, min(B, (i + 1) * K)
                j = i % a.nbuf
                if i >= a.nbuf:
                    sq.wait_event(freed[j])
                L.net_quantize_input_f32(xf[lo:hi].data_ptr(), bufs[j].data_ptr(), hi - lo, C, T, scale, 0,
                                         sq.cuda_stream)
                ready[j].record(sq)
                sf.wait_event(ready[j])
                L.net_model_compute_batch_async(bufs[j].data_ptr(), logits[lo:hi].data_ptr(), hi - lo, 0, sf.cuda_stream)
                freed[j].record(sf)
            L.net_argmax_batch(logits.data_ptr(), cls.data_ptr(), B, 4, 0, sf.cuda_stream)
            done.record(sf)
            s0.wait_event(done)
            s0.wait_stream(sq)

        cls.zero_()
        pipe()
        torch.cuda.synchronize()
        ok = bool(torch.equal(cls, want))
        print(f"pipelined, chunk {K:6d} x {a.nbuf} buffers: {timed(pipe):.3f} ms per {B} trials, same classes: {ok}",
              flush=True)


if __name__ == "__main__":
    main()

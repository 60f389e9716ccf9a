#!/usr/bin/env python3
"""Throughput of the steps either side of the path, one MI355X.

The bar is the same as for the forward's bench line: HIP events on the launch stream, inputs
resident in HBM, algorithmic bytes / kernel time against the 8 TB/s HBM peak.  One JSON line per
step, at config B's shape (65,536 trials of 22 x 1125):

  quantize_f32   net_quantize_input_f32: float32 [B][C][T] -> int8 [B][stride]
                 (reads 4 C T B, writes stride B bytes)
  quantize_f64   net_quantize_input_f64: float64 input (reads 8 C T B)
  pack_i8        net_pack_trials_i8: int8 [B][C][T] -> [B][stride] (the transpose alone)
  argmax         net_argmax_batch: int8 [B][4] -> int32 [B] (B = 2^24 as well, where it is not
                 launch-bound)
  copy_ref       torch copy_ of the int8 trials: the read + write yardstick for the two above
  chain_f32      float32 input -> quantiser -> fused forward -> argmax, per trial

    python tools/bench_steps.py [--steps 20] [--warmup 3] [--lib tools/libX_diag.so] [--only quantize_f32,pack_i8]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet import lib  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402

PEAK_GBS = 8000.0


def timed(fn, steps, warmup, stream):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / steps  # ms


def line(step, ms, nbytes, B, note):
    gbs = nbytes / (ms * 1e-3) / 1e9
    return {"step": step, "avg_kernel_ms": ms, "trials": B, "trials_per_s": B / (ms * 1e-3),
            "bytes_per_launch": nbytes, "achieved_GBs": gbs, "peak_GBs": PEAK_GBS, "frac": gbs / PEAK_GBS,
            "note": note}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--lib", default=None, help="a library variant (tools/build_diag.sh) instead of the in-tree one")
    ap.add_argument("--only", default=None, help="comma-separated steps to run (default: all)")
    a = ap.parse_args()
    if a.lib:
        lib.load(os.path.abspath(a.lib))
    want = set(a.only.split(",")) if a.only else None
    run = lambda name: want is None or name in want  # noqa: E731
    C, T, B = 22, 1125, a.B
    ps = ParamSet.synthetic(seed=1)
    lib.params_load(ps)
    stride = lib.trial_stride()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    out = []

    xf = torch.randn((B, C, T), dtype=torch.float32, device=dev, generator=g) * 50.0
    scale = 200.0
    y = torch.empty((B, stride), dtype=torch.int8, device=dev)
    L = lib.load()
    f32 = lambda: L.net_quantize_input_f32(xf.data_ptr(), y.data_ptr(), B, C, T, ctypes_float(scale), 0,  # noqa: E731
                                           st.cuda_stream)
    if run("quantize_f32"):
        ms = timed(f32, a.steps, a.warmup, st)
        out.append(line("quantize_f32", ms, B * (4 * C * T + stride), B,
                        "reads the float32 trials, writes the batched int8 layout (pads included)"))

    x8 = torch.randint(-128, 128, (B, C, T), dtype=torch.int8, device=dev, generator=g)
    if run("copy_ref"):  # yardstick: the runtime's device-to-device copy of the same int8 bytes
        yc = torch.empty((B, C * T), dtype=torch.int8, device=dev)
        cp = lambda: yc.view(B, C, T).copy_(x8)  # noqa: E731
        ms = timed(cp, a.steps, a.warmup, st)
        out.append(line("copy_ref", ms, 2 * B * C * T, B, "torch copy_ of the int8 trials (read + write): the "
                        "practical ceiling of a read-once write-once kernel"))
        del yc
    pk = lambda: L.net_pack_trials_i8(x8.data_ptr(), y.data_ptr(), B, C, T, 0, st.cuda_stream)  # noqa: E731
    if run("pack_i8"):
        ms = timed(pk, a.steps, a.warmup, st)
        out.append(line("pack_i8", ms, B * (C * T + stride), B, "channel-major int8 -> [T][C] trial layout"))
    del x8

    z = torch.empty((B, 4), dtype=torch.int8, device=dev)
    cls = torch.empty((B,), dtype=torch.int32, device=dev)

    def chain():
        L.net_quantize_input_f32(xf.data_ptr(), y.data_ptr(), B, C, T, ctypes_float(scale), 0, st.cuda_stream)
        L.net_model_compute_batch_async(y.data_ptr(), z.data_ptr(), B, 0, st.cuda_stream)
        L.net_argmax_batch(z.data_ptr(), cls.data_ptr(), B, 4, 0, st.cuda_stream)

    if run("chain_f32"):
        ms = timed(chain, a.steps, a.warmup, st)
        out.append(line("chain_f32", ms, B * (4 * C * T + 4), B,
                        "float32 trials -> quantiser -> fused forward -> argmax; bytes = the float input "
                        "and the class ids (intermediates count 0)"))
    del xf

    xd = torch.randn((B // 2, C, T), dtype=torch.float64, device=dev, generator=g) * 50.0
    f64 = lambda: L.net_quantize_input_f64(xd.data_ptr(), y.data_ptr(), B // 2, C, T, ctypes_double(scale), 0,  # noqa: E731
                                           st.cuda_stream)
    if run("quantize_f64"):
        ms = timed(f64, a.steps, a.warmup, st)
        out.append(line("quantize_f64", ms, (B // 2) * (8 * C * T + stride), B // 2,
                        "float64 trials (half the batch, the same bytes as float32)"))
    del xd

    for nb in ((B, 1 << 24) if run("argmax") else ()):
        zz = torch.randint(-128, 128, (nb, 4), dtype=torch.int8, device=dev, generator=g)
        cc = torch.empty((nb,), dtype=torch.int32, device=dev)
        am = lambda: L.net_argmax_batch(zz.data_ptr(), cc.data_ptr(), nb, 4, 0, st.cuda_stream)  # noqa: E731
        ms = timed(am, a.steps, a.warmup, st)
        out.append(line("argmax", ms, nb * (4 + 4), nb, f"{nb} trials of 4 logits"))

    for o in out:
        print(json.dumps(o), flush=True)


def ctypes_float(v):
    import ctypes
    return ctypes.c_float(v)


def ctypes_double(v):
    import ctypes
    return ctypes.c_double(v)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Single-thread speed of the CPU oracle (the bench's cpu_baseline code) built for different ISA
levels: the shipped -march=x86-64-v3 build against AVX-512 builds given on the command line.
Diagnostic; picks the build the CPU baseline should use on this host."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
import oracle  # noqa: E402  (test infrastructure)
from mibminet.params import ParamSet, pack_trials  # noqa: E402


def main():
    ps = ParamSet.synthetic(seed=1)
    x = pack_trials(np.random.default_rng(0).integers(-128, 128, size=(96, 22, 1125)))
    ref = None
    for path in [oracle._LIB_PATH] + sys.argv[1:]:
        L = ctypes.CDLL(os.path.abspath(path))
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.or_model_compute_batch.argtypes = [vp, vp, sz, vp, sz, i]
        oracle._lib = L
        co = oracle.COracle(ps)
        co.batch(x[:4], nthreads=1)
        t = time.perf_counter()
        y = co.batch(x, nthreads=1)
        dt = time.perf_counter() - t
        ref = y if ref is None else ref
        print(f"{os.path.basename(path):28s} {x.shape[0] / dt:8.0f} trials/s, 1 thread, same logits: {np.array_equal(y, ref)}")


if __name__ == "__main__":
    main()

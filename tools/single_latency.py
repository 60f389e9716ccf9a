#!/usr/bin/env python3
"""Host-side latency of the reference's single-trial entry point net_model_compute (host buffers:
copy in, one fused-kernel launch over one trial, copy out), the way a real-time BCI host calls it
once per trial.  Diagnostic; prints the median and the 10/90 % points over N calls."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))
from mibminet import lib  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402


def main(n=2000):
    if len(sys.argv) > 2 and sys.argv[1] == "--lib":  # another build (tools/build_base.sh)
        lib.load(os.path.abspath(sys.argv[2]))
    ps = ParamSet.synthetic(seed=1)
    lib.params_load(ps)
    d = ps.dims
    rng = np.random.default_rng(0)
    x = rng.integers(-128, 128, size=(d.T, d.C_ALIGN)).astype(np.int8)
    x[:, d.C:] = 0
    L = lib.load()
    y = np.empty(d.N, np.int8)
    for _ in range(50):
        L.net_model_compute(x.ctypes.data, y.ctypes.data)
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        L.net_model_compute(x.ctypes.data, y.ctypes.data)
        ts.append(time.perf_counter() - t0)
    assert L.net_last_error() == 0
    ts = np.array(ts) * 1e6
    print(f"net_model_compute: median {np.median(ts):.1f} us, p10 {np.percentile(ts, 10):.1f}, "
          f"p90 {np.percentile(ts, 90):.1f}, p99 {np.percentile(ts, 99):.1f} ({n} calls)")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Transient-corruption stress check (diagnostic): repeats the GPU paths many times and counts
outputs that differ from the expected ones.

  1. net_layer1 (k_layer stage 1) on the stress fixture, N1 calls, against the fixture's y1;
  2. the fused batch kernel on B trials, N2 launches, each output compared with the oracle's
     logits (computed once on the CPU for the same inputs).

    python tools/stress.py [--lib path] [--n1 2000] [--n2 200] [--B 65536]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mi-bminet_amd"), ROOT]
import oracle  # noqa: E402
from mibminet import lib  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n1", type=int, default=2000)
    ap.add_argument("--n2", type=int, default=200)
    ap.add_argument("--B", type=int, default=65536)
    a = ap.parse_args()
    if a.lib:
        lib.load(os.path.abspath(a.lib))
    f = np.load(os.path.join(ROOT, "tests/golden/fixture_b22_stress.npz"))
    ps = ParamSet.from_blob(f["blob"].tobytes())
    lib.params_load(ps)
    xa = oracle.to_tc_align(f["x"][0], ps.dims.C_ALIGN)
    t0 = time.time()
    bad1 = 0
    for i in range(a.n1):
        y1 = lib.net_layer1(xa)
        nb = int((y1 != f["y1"]).sum())
        if nb:
            bad1 += 1
            if bad1 <= 5:
                w = np.argwhere(y1 != f["y1"])
                print(f"layer1 call {i}: {nb} bytes differ, first {w[:4].tolist()}", flush=True)
    print(f"layer1: {bad1} of {a.n1} calls wrong ({time.time() - t0:.1f} s)", flush=True)

    for stress in (True, False):
        ps = ParamSet.synthetic(seed=7, stress=stress)
        lib.params_load(ps)
        stride = lib.trial_stride()
        g = torch.Generator(device="cuda:0").manual_seed(11)
        x = torch.randint(-128, 128, (a.B, stride), dtype=torch.int8, device="cuda:0", generator=g)
        x[:, 22 * 1125:] = 0
        want = oracle.COracle(ps).batch(x.cpu().numpy(), nthreads=min(16, os.cpu_count() or 1))
        want_t = torch.from_numpy(want).to("cuda:0")
        y = torch.empty((a.B, 4), dtype=torch.int8, device="cuda:0")
        bad2 = 0
        t0 = time.time()
        for i in range(a.n2):
            y.fill_(0x55)
            lib.model_compute_batch(x.data_ptr(), y.data_ptr(), a.B)
            torch.cuda.synchronize()
            nb = int((y != want_t).any(dim=1).sum())
            if nb:
                bad2 += 1
                if bad2 <= 5:
                    rows = torch.nonzero((y != want_t).any(dim=1)).flatten()[:4].tolist()
                    print(f"batch launch {i}: {nb} trials differ, first {rows}", flush=True)
        print(f"batch (stress={stress}): {bad2} of {a.n2} launches wrong ({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()

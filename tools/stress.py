#!/usr/bin/env python3
"""Transient-corruption stress check (diagnostic): repeats the GPU paths many times and counts
outputs that differ from the expected ones.

  1. net_layer1 (k_layer stage 1) on the stress fixture, N1 calls, against the fixture's y1;
  2. the fused batch kernel on B trials, N2 launches per parameter mode.  The inputs are NB
     distinct seeded batches (the oracle's logits computed once per batch on the CPU); launch i
     runs batch i % NB under a fresh random trial permutation (drawn on the device), so every
     launch maps different trials to different workgroups and prefetch slots, and is compared
     with the oracle's logits permuted the same way.

    python tools/stress.py [--lib path] [--n1 2000] [--n2 200] [--nb 8] [--B 65536] [--layout ct] [--cfg c64]

  --layout ct stresses net_model_compute_batch_ct instead: the batches are channel-major
  [B][C][T] (the oracle gets the same trials transposed).  --layout f32 stresses
  net_model_compute_batch_f32 on float32 batches against the two-pass GPU chain
  (net_quantize_input_f32 + the time-major forward, which the GPU tests pin to the oracle).
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
    ap.add_argument("--nb", type=int, default=8, help="distinct input batches per parameter mode")
    ap.add_argument("--layout", default="tc", choices=("tc", "ct", "f32"))
    ap.add_argument("--cfg", default="b22", choices=("b22", "c64", "p64", "g19", "g38", "p64l"),
                    help="geometry of the batch stress (g19 / g38 / p64l: the general kernels)")
    ap.add_argument("--force-general", action="store_true",
                    help="run the compiled geometries on the general kernels (mibminet_test_force_general)")
    ap.add_argument("--variants", default="canonical",
                    help="comma list of build variants to stress: canonical, plain_bn, clip_balanced")
    ap.add_argument("--extreme", action="store_true",
                    help="ParamSet.synthetic_extreme sets (the exact-division kernels) instead of synthetic")
    a = ap.parse_args()
    if a.lib:
        lib.load(os.path.abspath(a.lib))
    if a.force_general:
        lib.force_general(True)
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

    modes = [(v, st) for v in a.variants.split(",") for st in ((False,) if a.extreme else (True, False))]
    for variant, stress in modes:
        gC, gT, gN = {"b22": (22, 1125, 4), "c64": (64, 1000, 4), "p64": (64, 480, 4), "g19": (19, 1125, 3),
                      "g38": (38, 480, 2), "p64l": (64, 960, 4)}[a.cfg]
        if a.extreme:
            ps = ParamSet.synthetic_extreme(7, reorder_bn=variant != "plain_bn",
                                            clip_balanced=variant == "clip_balanced", C=gC, T=gT, N=gN)
        else:
            ps = ParamSet.synthetic(seed=7, stress=stress, reorder_bn=variant != "plain_bn",
                                    clip_balanced=variant == "clip_balanced", C=gC, T=gT, N=gN)
        lib.params_load(ps)
        stride = lib.trial_stride()
        g = torch.Generator(device="cuda:0").manual_seed(11 + stress)
        xs, wants = [], []
        t0 = time.time()
        C, T = ps.dims.C, ps.dims.T
        for k in range(a.nb):
            if a.layout == "f32":
                xf = torch.randn((a.B, C, T), dtype=torch.float32, device="cuda:0", generator=g)
                xs.append(xf.view(a.B, C * T))
                wants.append(lib.forward_torch(lib.quantize_input_torch(xf, 3.0)).clone())
                continue
            if a.layout == "ct":
                xc = torch.randint(-128, 128, (a.B, C * T), dtype=torch.int8, device="cuda:0", generator=g)
                x = torch.zeros((a.B, stride), dtype=torch.int8, device="cuda:0")
                x[:, : C * T] = xc.view(a.B, C, T).transpose(1, 2).reshape(a.B, C * T)
                xs.append(xc)
            else:
                x = torch.randint(-128, 128, (a.B, stride), dtype=torch.int8, device="cuda:0", generator=g)
                x[:, C * T:] = 0
                xs.append(x)
            want = oracle.COracle(ps).batch(x.cpu().numpy(), nthreads=min(16, os.cpu_count() or 1))
            wants.append(torch.from_numpy(want).to("cuda:0"))
            del x
        print(f"oracle on {a.nb} x {a.B} trials: {time.time() - t0:.1f} s", flush=True)
        xp = torch.empty_like(xs[0])
        y = torch.empty((a.B, ps.dims.N), dtype=torch.int8, device="cuda:0")
        bad2 = 0
        t0 = time.time()
        for i in range(a.n2):
            k = i % a.nb
            perm = torch.randperm(a.B, device="cuda:0", generator=g)
            torch.index_select(xs[k], 0, perm, out=xp)
            y.fill_(0x55)
            if a.layout == "f32":
                rc = lib.load().net_model_compute_batch_f32(xp.data_ptr(), y.data_ptr(), a.B, 3.0, 0, None)
                assert rc == 0, rc
            elif a.layout == "ct":
                rc = lib.load().net_model_compute_batch_ct(xp.data_ptr(), y.data_ptr(), a.B, 0, None)
                assert rc == 0, rc
            else:
                lib.model_compute_batch(xp.data_ptr(), y.data_ptr(), a.B)
            torch.cuda.synchronize()
            bad = (y != wants[k][perm]).any(dim=1)
            nb = int(bad.sum())
            if nb:
                bad2 += 1
                if bad2 <= 5:
                    rows = torch.nonzero(bad).flatten()[:4].tolist()
                    print(f"batch launch {i}: {nb} trials differ, first {rows}", flush=True)
        print(f"batch ({a.layout}, {a.cfg}{' general' if a.force_general or a.cfg[0] == 'g' or a.cfg == 'p64l' else ''}, {variant}, {'extreme' if a.extreme else f'stress={stress}'}): {bad2} of {a.n2} launches wrong, {a.n2 * a.B:.3g} trials checked, "
              f"{a.nb * a.B} distinct ({time.time() - t0:.1f} s)", flush=True)

if __name__ == "__main__":
    main()

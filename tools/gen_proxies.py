#!/usr/bin/env python3
"""Builds timing proxies of the general kernels (results wrong) from scratch copies in /tmp/gd:
tools/probebin_gd<name>, each tools/probe.hip with -DMIB_STAMPS over a patched forward_gen.hpp."""
import os, shutil, subprocess, sys
ROOT = "/root/repo"
V = {
    "base": [],
    "nol1rd": [("if constexpr (ST) raw[u] = l1_fetch_lds<false>(src, blk);",
                "if constexpr (ST) raw[u] = (v4i){blk, lane, C, T};")],
    "nol1st": [("*(unsigned*)(y1 + j * y1s + 32 + t0) = sat4(y[0], y[1], y[2], y[3]);",
                "if (y[0] == 12345) *(unsigned*)(y1 + j * y1s + 32 + t0) = sat4(y[0], y[1], y[2], y[3]);")],
    "nol2rd": [("bs[fi][s] = *(const v4i*)(y1 + (2 * wave + fi) * y1s + 1024 * mt + 32 * n + 16 * h + 32 * s);",
                "bs[fi][s] = (v4i){mt, n, h, s};"),
               ("for (int s = 0; s < 2; s++) bt[fi][s] = *(const v4i*)(y1 + (2 * wave + fi) * y1s + p0 + 64 * s + 16 * g);",
                "for (int s = 0; s < 2; s++) bt[fi][s] = (v4i){p0, s, g, fi};")],
    "nol3rd": [("const v4i b = *(const v4i*)(src + step * t);", "const v4i b = (v4i){t, step, lane, 0};")],
    "nol3st": [("if (u0 + q < T8) y3[16 * (u0 + q) + f] = (int8_t)clampq(y, LO);",
                "if (y == 12345) y3[16 * (u0 + q) + f] = (int8_t)clampq(y, LO);")],
    "nol4rd": [("const v4i a = *(const v4i*)(y3 + 16 * (64 * p + 32 * h + n));", "const v4i a = (v4i){p, h, n, 0};")],
    "nodma": [("if (ST && bn < B) stage_trial(", "if (false) stage_trial(")],
}
names = sys.argv[1:] or list(V)
procs = []
for name in names:
    d = f"/tmp/gd/{name}"
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(f"{ROOT}/mi-bminet_amd/csrc", f"{d}/mi-bminet_amd/csrc")
    shutil.copytree(f"{ROOT}/include", f"{d}/include")
    os.makedirs(f"{d}/tools")
    shutil.copy(f"{ROOT}/tools/probe.hip", f"{d}/tools/probe.hip")
    p = f"{d}/mi-bminet_amd/csrc/forward_gen.hpp"
    s = open(p).read()
    for a, b in V[name]:
        assert a in s, (name, a)
        s = s.replace(a, b)
    open(p, "w").write(s)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-function",
           "-mllvm", "-disable-promote-alloca-to-lds", "-DMIB_STAMPS", "-o", f"{ROOT}/tools/probebin_gd{name}",
           f"{d}/tools/probe.hip"]
    procs.append((name, subprocess.Popen(cmd)))
for name, pr in procs:
    print(name, pr.wait())

#!/usr/bin/env python3
"""In-kernel float quantiser of a library build (mibminet_test_quantize_f32) against the two-pass
quantiser (net_quantize_input_f32) on all 2^32 float32 bit patterns (diagnostic: checks -D
variants of the fused float path before one becomes the shipped form; tests/test_gpu_f32.py
does the same for the shipped library).

    python tools/fq_check.py tools/libX_diag.so [scale ...]
"""
import ctypes
import os
import sys

import torch


def main():
    L = ctypes.CDLL(os.path.abspath(sys.argv[1]), mode=ctypes.RTLD_LOCAL)
    L.mibminet_test_quantize_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_float,
                                              ctypes.c_int, ctypes.c_void_p]
    L.net_quantize_input_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    scales = [float(s) for s in sys.argv[2:]] or [1.0, 1.7, 2.0 ** -60, 2.0 ** 60]
    n, T = 1 << 28, 1 << 14
    got = torch.empty(n, dtype=torch.int8, device="cuda")
    want = torch.empty(n, dtype=torch.int8, device="cuda")
    total = 0
    for scale in scales:
        bad = 0
        for chunk in range(16):
            x = torch.arange(chunk * n, (chunk + 1) * n, dtype=torch.int64, device="cuda").to(torch.int32)
            x = x.view(torch.float32)
            assert L.mibminet_test_quantize_f32(x.data_ptr(), got.data_ptr(), n, scale, 0, None) == 0
            assert L.net_quantize_input_f32(x.data_ptr(), want.data_ptr(), n // T, 1, T, scale, 0, None) == 0
            torch.cuda.synchronize()
            d = got != want
            if bool(d.any()):
                i = int(torch.nonzero(d)[0])
                bad += int(d.sum())
                print(f"  scale {scale}: bits {chunk * n + i:#010x} got {int(got[i])} want {int(want[i])}")
        print(f"{os.path.basename(sys.argv[1])} scale {scale}: {bad} of 2^32 differ", flush=True)
        total += bad
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()

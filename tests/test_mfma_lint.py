"""Device-assembly check of the fused kernels (CPU only: hipcc cross-compiles gfx950).

tools/mfma_lint.py flags inline-asm instructions that write a register of an earlier MFMA's
destination before anything has read it.  The compiler's hazard checks do not cover inline asm,
so the MFMA's write-back can land after the asm result; round 2 hit this in layer 3 (DESIGN.md
§3).  The build must show none.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_inline_asm_write_into_pending_mfma_dst(tmp_path):
    asm = tmp_path / "mibminet.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function",
                    "-mllvm", "-disable-promote-alloca-to-lds", "--cuda-device-only", "-S", "-o", str(asm),
                    os.path.join(ROOT, "mi-bminet_amd", "csrc", "mibminet.hip")],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mfma_lint.py"), str(asm)],
                       check=True, capture_output=True, text=True)
    hazards = [l for l in r.stdout.splitlines() if "asm write into pending dst" in l]
    assert not hazards, "\n".join(hazards)

"""The plain-C host (examples/c_host/net_host.c): the library used from C through the C ABI
alone, as the reference's own C callers use net_model_compute (test/cl/net/model/cluster.c:40-49
compares the logits with the golden model's; `net_host check` does the same against the oracle).
"""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from mibminet.params import ParamSet

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "c_host")
BIN = os.path.join(EX, "net_host")


@pytest.fixture(scope="module")
def net_host():
    subprocess.run(["make", "-s", "-C", EX], check=True)
    return BIN


def test_builds_and_prints_usage(net_host):
    r = subprocess.run([net_host], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("C,T,rb", [(22, 1125, True), (64, 1000, True), (22, 1125, False)])
def test_c_host_check(gpu, net_host, tmp_path, C, T, rb):
    ps = ParamSet.synthetic(seed=C + T, C=C, T=T, stress=True, reorder_bn=rb)
    d = ps.dims
    n = 24
    rng = np.random.default_rng(C)
    x = np.stack([oracle.to_tc_align(rng.integers(-128, 128, size=(C, T)), d.C_ALIGN) for _ in range(n)])
    co = oracle.COracle(ps)
    want = np.stack([co.model(xi) for xi in x])
    (tmp_path / "p.blob").write_bytes(ps.to_blob())
    (tmp_path / "x.bin").write_bytes(x.astype(np.int8).tobytes())
    (tmp_path / "want.bin").write_bytes(want.astype(np.int8).tobytes())
    r = subprocess.run([net_host, "check", str(tmp_path / "p.blob"), str(tmp_path / "x.bin"),
                        str(tmp_path / "want.bin"), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
    assert f"net_model_compute_batch_ct: 0 of {n} trials differ" in r.stdout
    # a wrong expectation is reported as a failure
    bad = want.copy()
    bad[3, 0] ^= 1
    (tmp_path / "bad.bin").write_bytes(bad.astype(np.int8).tobytes())
    r = subprocess.run([net_host, "check", str(tmp_path / "p.blob"), str(tmp_path / "x.bin"),
                        str(tmp_path / "bad.bin"), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "1 of 24 trials differ" in r.stdout


@pytest.mark.gpu
def test_c_host_bench(gpu, net_host, tmp_path):
    (tmp_path / "p.blob").write_bytes(ParamSet.synthetic(seed=1).to_blob())
    r = subprocess.run([net_host, "bench", str(tmp_path / "p.blob"), "65536", "20"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    m = re.search(r"([0-9.e+]+) trials/s", r.stdout)
    assert m and float(m.group(1)) > 1e7, r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["net_b22", "net_g19"])
def test_c_host_linked_net_h(gpu, tmp_path, name):
    """The C host linked with a generated net.c (the reference's weight globals, examples/c_host/
    make_nets.py) loads it through net_params_load_arrays (no blob file) and matches the oracle on
    net_model_compute, net_model_compute_batch and net_model_compute_batch_ct."""
    import sys
    sys.path.insert(0, EX)
    import make_nets

    subprocess.run(["make", "-s", "-C", EX], check=True)
    ps = make_nets.param_set(name)
    d = ps.dims
    n = 20
    rng = np.random.default_rng(d.C)
    x = np.stack([oracle.to_tc_align(rng.integers(-128, 128, size=(d.C, d.T)), d.C_ALIGN) for _ in range(n)])
    co = oracle.COracle(ps)
    want = np.stack([co.model(xi) for xi in x])
    (tmp_path / "x.bin").write_bytes(x.astype(np.int8).tobytes())
    (tmp_path / "want.bin").write_bytes(want.astype(np.int8).tobytes())
    exe = os.path.join(EX, "net_host_" + name.split("_")[1])
    r = subprocess.run([exe, "check", "-", str(tmp_path / "x.bin"), str(tmp_path / "want.bin"), str(n)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "parameters: linked net.c" in r.stdout and "ok" in r.stdout
    assert f"net_model_compute_batch_ct: 0 of {n} trials differ" in r.stdout

"""bench.py's multi-rank branch on the CPU (static split, no collectives): two
ranks under torch.distributed.run coordinate over a gloo group only, each times its own steps, and
rank 0 prints one JSON line with the world size, the backend and every rank's record.  The step is
a host stand-in (MIB_BENCH_STUB=1): no GPU and no library compute."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_multi_rank_gloo_only():
    env = dict(os.environ, MIB_BENCH_STUB="1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--settle", "0",
           "--batch", "64", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["stub"] and out["n_gpus"] == 2 and out["scaling"] == "weak"
    assert out["ranks"]["world_size"] == 2
    assert out["ranks"]["backend"] == "gloo"
    assert [p["rank"] for p in out["ranks"]["per_rank"]] == [0, 1]
    assert out["config"]["global_batch"] == 128 and out["value"] > 0
    # the elapsed time reported is the slowest rank's
    assert abs(out["ms_per_step"] - max(p["elapsed_s"] for p in out["ranks"]["per_rank"]) / 3 * 1e3) < 1e-6
    assert "nccl" not in r.stdout + r.stderr.lower()
    assert out["parity"]["mismatches"] == 0 and out["parity"]["checked"] == 64


def _stub_run(extra_env=None, *args):
    env = dict(os.environ, MIB_BENCH_STUB="1", OMP_NUM_THREADS="1", **(extra_env or {}))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--settle", "0",
           "--batch", "32", "--no-cpu-baseline", *args]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)


def test_bench_parity_field_and_failure_exit():
    """The headline line carries "parity" (trials checked against the oracle, mismatches); a
    mismatch prints the line and then exits non-zero (stub stand-in, CPU)."""
    for layout, cfg in (("tc", "b22"), ("ct", "g38"), ("f32", "b22")):
        r = _stub_run(None, "--layout", layout, "--config", cfg)
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert out["parity"]["checked"] == 32 and out["parity"]["mismatches"] == 0
    r = _stub_run({"MIB_BENCH_STUB_CORRUPT": "1"})
    assert r.returncode != 0
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["parity"]["mismatches"] == 1 and out["parity"]["first_bad"] == [16]
    assert "differ from the oracle" in r.stderr

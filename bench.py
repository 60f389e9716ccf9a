#!/usr/bin/env python3
"""Benchmark of the MI355X int8 MI-BMInet forward (BASELINE.json metric).

One "step" = one fused forward pass (one kernel launch) over a batch of 65,536 synthetic
22-channel x 1125-sample int8 trials already resident in HBM (BASELINE config B; with --gpus N
each rank owns its own 65,536-trial shard: config E's static split, weak scaling, no collectives).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config b22|c64|d22|p64|g19|g38|p64l] [--batch B]

For N > 1 launch under ``torch.distributed.run`` (one process per GPU); rank 0 prints ONE JSON
line.  ``value`` = trials processed by all ranks / max-over-ranks wall time of the K timed steps.
The ranks coordinate over a gloo (host) group only: the start barrier, the max-of-elapsed
reduction and the per-rank record.  The data path has no collective, so no RCCL
group is ever created, and nothing collective runs inside the K timed steps: each rank times its
own steps (host clock around them, HIP events on its launch stream), then the ranks reduce.
``roofline.achieved`` = algorithmic bytes per launch (input 22*1125 B + 4 B logits per trial) /
average kernel duration from HIP events on the launch stream.  ``cpu_baseline`` times the C
restatement of the reference forward (oracle/, kind "port") on the host cores (rank 0, N = 1),
and its logits on that sample are compared with the timed batch's: ``parity`` = trials checked and
mismatches; any mismatch makes the run exit non-zero (after printing the line).  Without a timed
baseline (--no-cpu-baseline, or N > 1) the oracle still checks the whole batch (rank 0's shard),
untimed, after the timed steps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mi-bminet_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mibminet import lib  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402

METRIC = "EEG trials/sec (int8, 22ch×1125) at batch 65536; bit-exact logits"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
CONFIGS = {
    "b22": dict(C=22, T=1125, wbits=8, name="B: 22ch x 1125 int8, 4-class"),
    "c64": dict(C=64, T=1000, wbits=8, name="C: 64ch x 1000 int8, 4-class"),
    "d22": dict(C=22, T=1125, wbits=4, name="D: 22ch x 1125, int4 weights / int8 acts"),
    "p64": dict(C=64, T=480, wbits=8, name="PhysioNet MMMI: 64ch x 480 int8, 4-class (not a BASELINE config)"),
    # geometries without a compiled kernel: the run-time-dimension kernels (forward_gen.hpp)
    "g19": dict(C=19, T=1125, wbits=8, N=3, name="channel-selected 19ch x 1125 int8, 3-class (general kernels)"),
    "g38": dict(C=38, T=480, wbits=8, N=2, name="PhysioNet channel-selected 38ch x 480 int8, 2-class (general kernels)"),
    "p64l": dict(C=64, T=960, wbits=8, N=4, name="PhysioNet MMMI 6 s window: 64ch x 960 int8, 4-class (general kernels)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="trials per GPU")
    ap.add_argument("--config", default="b22", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--variant", default="canonical", choices=("canonical", "plain_bn", "clip_balanced"),
                    help="build variant the parameter blob selects: the canonical -DREORDER_BN build, the "
                         "plain-BN branches (layer2.c:139-210, layer4.c:91-133) or golden-model balanced clipping")
    ap.add_argument("--layout", default="tc", choices=("tc", "ct", "f32"),
                    help="input layout: tc = time-major batched trials [B][stride] (net_model_compute_batch), "
                         "ct = channel-major [B][C][T] (net_model_compute_batch_ct, transposed inside the kernel), "
                         "f32 = float32 EEG [B][C][T] (net_model_compute_batch_f32, quantised inside the kernel)")
    ap.add_argument("--params", default="synthetic", choices=("synthetic", "extreme", "rails"),
                    help="synthetic: calibrated seeded weights (the benchmark set, float requant kernels); "
                         "extreme: requant factors and offsets far outside the float envelope "
                         "(ParamSet.synthetic_extreme, the exact integer-division kernels); "
                         "rails: the same with only constant (rail / zero / suppressed) filters out of "
                         "the envelope, which the loader folds (float kernels)")
    ap.add_argument("--force-general", action="store_true",
                    help="run the run-time-dimension kernels even on a compiled geometry (comparison)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle", type=float, default=0.25,
                    help="seconds of untimed launches before the warmup steps (GPU clock ramp)")
    ap.add_argument("--per-launch-events", action="store_true",
                    help="bracket every launch with its own HIP events (diagnostic; adds idle gaps)")
    ap.add_argument("--cpu-seconds", type=float, default=25.0, help="target CPU-baseline wall time")
    ap.add_argument("--pcie", action="store_true",
                    help="also time the host-buffer path (pinned H2D + forward + D2H); reported as "
                         "'pcie_inclusive', never as value")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


# MIB_BENCH_STUB=1 (CPU tests only, tests/test_bench_cpu.py): the multi-rank bookkeeping with a
# stand-in step on the host and no device or library compute; its lines are marked "stub" and
# are never bench results.
STUB = os.environ.get("MIB_BENCH_STUB") == "1"


def _cpu_quota():
    """CPUs granted by the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs), or None if unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def cpu_baseline(ps, x_dev, seconds):
    """Times the oracle's C restatement of net_model_compute on a bounded sample of the same
    workload (rank 0, N = 1 only): (ii) all host cores this process may use, and (i) one core
    (SURVEY §8(d)).  "All cores" = one pthread per CPU of the affinity mask, capped at the cgroup
    CPU quota when one is set: the GPU boxes show 256 CPUs in the mask but grant 16 CPUs of time,
    and 256 threads under a 16-CPU quota are throttled (measured: 5.0e4 trials/s against 9.2e4
    with 16 threads)."""
    sys.path.insert(0, ROOT)
    import oracle  # test infrastructure: only this leg of bench.py may use it

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    quota = _cpu_quota()
    usable = ncpu if quota is None else max(1, min(ncpu, int(quota + 0.999)))
    threads = max(1, int(os.environ.get("MIB_CPU_THREADS", usable)))
    co = oracle.COracle(ps)
    # calibrate on about a second of work (a short burst can exceed the quota within one period)
    calib = x_dev[: max(256, 4 * threads)].cpu().numpy()
    t0 = time.perf_counter()
    co.batch(calib, nthreads=threads)
    dt = max(time.perf_counter() - t0, 1e-6)
    if dt < 0.5:
        calib = x_dev[: min(x_dev.shape[0], int(calib.shape[0] * 1.0 / dt))].cpu().numpy()
        t0 = time.perf_counter()
        co.batch(calib, nthreads=threads)
        dt = max(time.perf_counter() - t0, 1e-6)
    per_trial = dt / calib.shape[0]
    want = max(8 * threads, int(seconds / per_trial))
    n = int(min(x_dev.shape[0], want))
    reps = max(1, min(64, want // n))  # the whole batch is cheaper than the target: repeat it
    sample = x_dev[:n].cpu().numpy()
    t0 = time.perf_counter()
    for _ in range(reps):
        logits = co.batch(sample, nthreads=threads)
    dt = time.perf_counter() - t0
    n *= reps
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    # (i) one core, on a smaller bounded sample (about a fifth of the time budget)
    t1 = time.perf_counter()
    co.batch(calib[:16], nthreads=1)
    per1 = max(time.perf_counter() - t1, 1e-6) / 16
    n1 = int(max(16, min(x_dev.shape[0], seconds / 5 / per1)))
    s1 = x_dev[:n1].cpu().numpy()
    t1 = time.perf_counter()
    co.batch(s1, nthreads=1)
    d1 = time.perf_counter() - t1
    # (ii') when a quota caps the thread count: also one thread per CPU of the whole affinity
    # mask, on a bounded sample (about a fifth of the budget at the quota-limited rate)
    mask = None
    if threads < ncpu and "MIB_CPU_THREADS" not in os.environ:
        nm = int(min(x_dev.shape[0], max(4 * ncpu, seconds / 5 / per_trial)))
        sm = x_dev[:nm].cpu().numpy()
        tm = time.perf_counter()
        co.batch(sm, nthreads=ncpu)
        dm = time.perf_counter() - tm
        mask = {"value": nm / dm, "unit": "trials/s", "threads": ncpu,
                "sample": f"{nm} trials, {ncpu} threads under a {quota}-CPU quota, {dm:.1f} s"}
    return logits, {"value": n / dt, "unit": "trials/s", "cores": threads, "kind": "port",
            "sample": f"{n} trials ({reps} pass(es) over the first {n // reps} trials) of the same synthetic batch, C restatement (oracle/oracle.c, -O3) "
                      f"of net_model_compute, {threads} host threads (one per usable CPU: affinity mask "
                      f"{ncpu}, cgroup quota {quota}) on {cpu}, {dt:.1f} s",
            "one_core": {"value": n1 / d1, "unit": "trials/s", "sample": f"{n1} trials, 1 thread, {d1:.1f} s"},
            "affinity_mask_threads": mask,
            "host_cpus": {"affinity": ncpu, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota,
                          "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}}


def oracle_logits(ps, x_dev, n):
    """The checker of the CPU leg when the baseline is not timed (--no-cpu-baseline, or N > 1: rank
    0's own shard): the oracle's logits of the first n trials, one thread per usable CPU."""
    sys.path.insert(0, ROOT)
    import oracle  # test infrastructure: the checker, never the thing measured

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    quota = _cpu_quota()
    threads = ncpu if quota is None else max(1, min(ncpu, int(quota + 0.999)))
    return oracle.COracle(ps).batch(x_dev[:n].cpu().numpy(), nthreads=threads)


def logit_parity(y_host, want):
    """Trials of the timed batch whose logits differ from the oracle's on the same trials
    (the reference's own exact-logit check around its timed call, test/cl/net/model/cluster.c:44-49)."""
    n = want.shape[0]
    bad = np.nonzero(np.any(y_host[:n] != want, axis=1))[0]
    return {"checked": int(n), "mismatches": int(bad.size), "first_bad": bad[:8].tolist(),
            "against": "oracle/oracle.c (C restatement of net_model_compute) on the first trials of the timed batch"}


def pcie_inclusive(x, y, B, device, sp, stream, reps=5):
    """Trials/s when the batch starts and ends in pinned host memory: H2D copy of the inputs,
    the forward, D2H copy of the logits, all on one stream (no overlap)."""
    xh = x.cpu().pin_memory()
    yh = torch.empty(y.shape, dtype=y.dtype).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(reps):
            x.copy_(xh, non_blocking=True)
            lib.model_compute_batch(x.data_ptr(), y.data_ptr(), B, device, sp)
            yh.copy_(y, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return {"value": B / dt, "unit": "trials/s", "ms_per_batch": dt * 1e3,
            "h2d_bytes": int(x.numel()), "note": "pinned host buffers, serial H2D + kernel + D2H"}


def main():
    a = parse()
    cfg = CONFIGS[a.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one rank per GPU)")
    dist = None
    if STUB:
        dev = torch.device("cpu")
    else:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1:
        # host-side coordination only (gloo): barriers, the max-of-elapsed reduction, the per-rank
        # record; several ranks may also share one GPU this way (tools/gloo_rehearsal.sh)
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://")

    kw = dict(C=cfg["C"], T=cfg["T"], weight_bits=cfg["wbits"], reorder_bn=a.variant != "plain_bn",
              clip_balanced=a.variant == "clip_balanced")
    if a.params in ("extreme", "rails"):
        ps = ParamSet.synthetic_extreme(a.seed, mids=6 if a.params == "extreme" else 0, N=cfg.get("N", 4), **kw)
    else:
        ps = ParamSet.synthetic(a.seed, N=cfg.get("N", 4), **kw)
    if a.force_general and not STUB:
        lib.force_general(True)
    lib.params_load(ps)
    info_p = {"path": "stub", "layer": 0, "filter": -1, "shape": -1} if STUB else lib.params_info()
    stride = lib.trial_stride()
    B = a.batch
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed * 1000 + rank)
    sync = (lambda: None) if STUB else (lambda: torch.cuda.synchronize(dev))
    C, T, N = cfg["C"], cfg["T"], ps.dims.N  # the logits' row length is the loaded set's
    if STUB:  # host int8 trials whatever the layout (no device, no library compute)
        x = torch.randint(-128, 128, (B, stride), dtype=torch.int8, generator=g)
    elif a.layout == "f32":
        # float EEG whose quantised values spread over the int8 range (scale = 3 sigma)
        xf = torch.randn((B, C, T), dtype=torch.float32, device=dev, generator=g)
        qscale = 3.0
        x = lib.quantize_input_torch(xf, qscale)  # the same trials as int8, time-major (CPU baseline)
        sync()
    elif a.layout == "ct":
        xc = torch.randint(-128, 128, (B, C, T), dtype=torch.int8, device=dev, generator=g)
        x = torch.zeros((B, stride), dtype=torch.int8, device=dev)  # the same trials, time-major
        x[:, : C * T] = xc.transpose(1, 2).reshape(B, C * T)         # (CPU baseline and --pcie)
    else:
        x = torch.randint(-128, 128, (B, stride), dtype=torch.int8, device=dev, generator=g)
        x[:, C * T:] = 0
    y = torch.empty((B, N), dtype=torch.int8, device=dev)
    stream = None if STUB else torch.cuda.current_stream(dev)
    sp = None if STUB else stream.cuda_stream
    ct_fn = lib.load().net_model_compute_batch_ct
    f32_fn = lib.load().net_model_compute_batch_f32

    def step():
        if STUB:
            y.copy_(x[:, :N])  # stand-in work on the host
        elif a.layout == "f32":
            rc = f32_fn(xf.data_ptr(), y.data_ptr(), B, qscale, local, sp)
            if rc:
                raise lib.NetError(rc, "net_model_compute_batch_f32")
        elif a.layout == "ct":
            rc = ct_fn(xc.data_ptr(), y.data_ptr(), B, local, sp)
            if rc:
                raise lib.NetError(rc, "net_model_compute_batch_ct")
        else:
            lib.model_compute_batch(x.data_ptr(), y.data_ptr(), B, local, sp)

    # settle (untimed, before the W warmup steps): from idle the GPU clock needs some tens of ms
    # of load to reach its steady state; without this the first ~50 ms run about 7 % slower
    # (measured: W = 5 -> 0.467 ms/step, W = 50 or 200 -> 0.436-0.439 ms/step on config B)
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < a.settle:
        for _ in range(20):
            step()
        sync()
    for _ in range(a.warmup):
        step()
    sync()
    if dist:
        dist.barrier()  # gloo, host side: every rank starts its K steps together
    sync()
    # HIP events on the launch stream bracket the K back-to-back launches (an event pair around
    # every launch leaves the GPU idle between launches: about +10 % per step on config B);
    # --per-launch-events keeps that mode for diagnostics
    nev = a.steps if a.per_launch_events else 1
    ev = None if STUB else [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                            for _ in range(nev)]
    t0 = time.perf_counter()
    if STUB:
        for i in range(a.steps):
            step()
    elif a.per_launch_events:
        for i in range(a.steps):
            ev[i][0].record(stream)
            step()
            ev[i][1].record(stream)
    else:
        ev[0][0].record(stream)
        for i in range(a.steps):
            step()
        ev[0][1].record(stream)
    sync()
    elapsed = time.perf_counter() - t0  # this rank's K steps; no collective inside
    if STUB:
        kernel_ms = [elapsed * 1e3 / a.steps]
    else:
        kernel_ms = ([s.elapsed_time(e) for s, e in ev] if a.per_launch_events
                     else [ev[0][0].elapsed_time(ev[0][1]) / a.steps])
    rank_avg_ms = float(np.mean(kernel_ms))
    per_rank = None
    if dist:
        # after the timed steps: the slowest rank's wall time (gloo, host tensors)
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed_max = float(t.item())
        # per-rank record (outside the timed region): which device, its kernel time and its wall time
        mine = {"rank": rank, "local_rank": local, "device": local, "kernel_ms": rank_avg_ms,
                "elapsed_s": elapsed, "trials": B}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        elapsed = elapsed_max

    failed = None
    info = {"grid": 0, "threads": 0, "lds_bytes": 0} if STUB else lib.launch_info(B, local, channel_major=a.layout != "tc")
    if rank == 0:
        # N > 1: the slowest rank's kernel average (each rank's is listed under "ranks")
        avg_kernel_s = (max(r["kernel_ms"] for r in per_rank) if per_rank else rank_avg_ms) / 1e3
        alg_bytes_trial = cfg["C"] * cfg["T"] * (4 if a.layout == "f32" else 1) + N
        achieved = alg_bytes_trial * B / avg_kernel_s / 1e9
        traffic = None
        try:
            # HBM bytes per launch measured by PMC counters for this config and batch
            # (tools/collect_profile.py), per config under "configs"
            tj = json.load(open(a.traffic_json))
            # (time-major under the config's key, other input layouts under "<config>_<layout>")
            key = a.config if a.layout == "tc" else f"{a.config}_{a.layout}"
            tc = tj.get("configs", {}).get(key, tj if tj.get("config") == key else {})
            if tc.get("batch") == B and a.variant == "canonical" and a.params == "synthetic" and not a.force_general:
                traffic = tc["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            pass
        value = world * B * a.steps / elapsed
        out = {
            "metric": (METRIC if a.config == "b22" and a.variant == "canonical" and a.layout == "tc" and a.params == "synthetic"
                       and not a.force_general
                       else f"EEG trials/sec ({cfg['name']}, {a.variant} build, {a.params} parameters, "
                            f"{'general kernels, ' if a.force_general else ''}"
                            f"{ {'ct': 'channel-major', 'f32': 'float32 channel-major', 'tc': 'time-major'}[a.layout]} "
                            f"input) at batch {B}"),
            "value": value,
            "unit": "trials/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "settle_s": a.settle,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int8",
            "data": "synthetic (uniform int8 EEG generated on device; seeded synthetic integer weights)",
            "config": {"workload": cfg["name"], "variant": a.variant, "C": cfg["C"], "T": cfg["T"], "batch_per_gpu": B,
                       "input_layout": {"ct": "[B][C][T] channel-major (net_model_compute_batch_ct)",
                                        "f32": "[B][C][T] float32, quantised in the kernel (net_model_compute_batch_f32)",
                                        "tc": "[B][T][C] time-major, 16-byte trial stride (net_model_compute_batch)"}[a.layout],
                       "global_batch": world * B, "weight_bits": cfg["wbits"],
                       "parallelism": f"dp{world} static batch split, no collectives",
                       "grid": info["grid"], "threads": info["threads"], "lds_bytes": info["lds_bytes"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ("gen::k_forward<%s> (C=%d, T=%d, N=%d at run time)" % (
                             {"tc": "TM", "ct": "CT", "f32": "F32"}[a.layout], C, T, N)
                             if info_p["path"] == "general" else
                             "k_forward<Cfg<%d,%d,RB=%d,CB=%d,CT=%d,FQ=%d,XR=%d>>" % (
                             cfg["C"], cfg["T"], a.variant != "plain_bn", a.variant == "clip_balanced",
                             a.layout != "tc", a.layout == "f32", info_p["path"] == "exact")),
                         "avg_kernel_ms": avg_kernel_s * 1e3,
                         "alg_bytes_per_launch": alg_bytes_trial * B},
            "cpu_baseline": None,
            "requant": "float (proven exact)" if info_p["path"] == "float" else "exact integer division",
            "kernel_path": info_p,
            "parity": None,
        }
        if dist:
            out["ranks"] = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                            "devices_visible": 0 if STUB else torch.cuda.device_count(), "per_rank": per_rank,
                            "note": "each rank times its own shard; value = all ranks' trials / max-over-ranks "
                                    "wall time; coordination over gloo (host) only, no RCCL"}
        if STUB:
            out["stub"] = "MIB_BENCH_STUB: host stand-in step, bookkeeping test only, not a measurement"
            yh = y.numpy().copy()
            if os.environ.get("MIB_BENCH_STUB_CORRUPT") == "1":
                yh[B // 2, 0] ^= 1  # the parity check's failure path (tests/test_bench_cpu.py)
            out["parity"] = logit_parity(yh, x[:, :N].numpy())
            out["parity"]["against"] = "stub stand-in"
        if a.pcie and not STUB:
            out["pcie_inclusive"] = pcie_inclusive(x, y, B, local, sp, stream)
        if world == 1 and not a.no_cpu_baseline and not STUB:
            want, out["cpu_baseline"] = cpu_baseline(ps, x, a.cpu_seconds)
            out["parity"] = logit_parity(y[: want.shape[0]].cpu().numpy(), want)
        elif not STUB:  # no timed baseline: the whole batch (rank 0's shard) is still checked
            want = oracle_logits(ps, x, B)
            out["parity"] = logit_parity(y.cpu().numpy(), want)
            if world > 1:
                out["parity"]["against"] += " (rank 0's shard)"
        print(json.dumps(out), flush=True)
        if out["parity"] and out["parity"]["mismatches"]:
            failed = "bench.py: the timed batch's logits differ from the oracle's on %d of %d trials" % (
                out["parity"]["mismatches"], out["parity"]["checked"])
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    if failed:
        raise SystemExit(failed)


if __name__ == "__main__":
    main()

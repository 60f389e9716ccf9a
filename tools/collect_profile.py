#!/usr/bin/env python3
"""Turns a tools/profile_round.sh output directory into the committed profile artefacts:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_<cfg>.csv      per-dispatch WRITE_SIZE / TCC_EA0_RDREQ_* (configs B, C, D)
  profiles/pmc_traffic.json         HBM bytes per launch per config (bench.py's roofline.traffic)
  profiles/<tag>_bench_*.json       the bench JSON lines

FETCH_SIZE is doubled (gfx950 tallies 128-B fabric reads at 64 B: MI355X_MICROARCH.md, HBM
section); WRITE_SIZE is taken as is.  Both counters report kB (1024 B).

    python tools/collect_profile.py gpurun_out/prof_r01 r01
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_forward"


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


def pmc_values(path, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if KERNEL in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(one(f"{src}/trace/**/*kernel_stats.csv"), f"{prof}/{tag}_kernel_stats.csv")
    g = glob.glob(f"{src}/trace_g19/**/*kernel_stats.csv", recursive=True)
    if g:  # the general kernels (config g19)
        shutil.copy(g[0], f"{prof}/{tag}_kernel_stats_g19.csv")
    for cfg in ("b22", "c64", "d22", "p64", "b22_ct", "c64_ct", "b22_f32", "g19", "g38", "p64l", "b22_extreme",
                "b22_rails"):
        p = f"{src}/bench_{cfg}.json"
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                open(f"{prof}/{tag}_bench_{cfg}.json", "w").write(lines[-1])
    fetch = pmc_values(one(f"{src}/pmc_fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    rcols = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
    # skip the first (warm-up) dispatch
    med = lambda v: sorted(v[1:] or v)[len(v[1:] or v) // 2]  # noqa: E731
    alg = {"b22": 22 * 1125 + 4, "c64": 64 * 1000 + 4, "d22": 22 * 1125 + 4,
           "b22_ct": 22 * 1125 + 4, "c64_ct": 64 * 1000 + 4, "b22_f32": 4 * 22 * 1125 + 4,
           "g19": 19 * 1125 + 3, "g38": 38 * 480 + 2, "p64l": 64 * 960 + 4}
    kern = {"b22": "k_forward<Cfg<22,1125,RB=1,CB=0>>", "c64": "k_forward<Cfg<64,1000,RB=1,CB=0>>",
            "d22": "k_forward<Cfg<22,1125,RB=1,CB=0>>", "b22_ct": "k_forward<Cfg<22,1125,RB=1,CB=0,CT=1>>",
            "c64_ct": "k_forward<Cfg<64,1000,RB=1,CB=0,CT=1>>", "b22_f32": "k_forward<Cfg<22,1125,RB=1,CB=0,CT=1,FQ=1>>",
            "g19": "gen::k_forward<TM,ST,RB,float,CB=0> (19x1125, N=3)", "g38": "gen::k_forward<TM,ST,RB,float,CB=0> (38x480, N=2)",
            "p64l": "gen::k_forward<TM,ST,RB,float,CB=0> (64x960, N=4)"}
    configs = {}
    for cfg in ("b22", "c64", "d22", "b22_ct", "c64_ct", "b22_f32", "g19", "g38", "p64l"):
        wf = glob.glob(f"{src}/pmc_write_{cfg}/**/*counter_collection.csv", recursive=True)
        rq = glob.glob(f"{src}/pmc_rdreq_{cfg}/**/*counter_collection.csv", recursive=True)
        if not (wf and rq):
            continue
        write = pmc_values(wf[0], "WRITE_SIZE")
        rvals = {c: pmc_values(rq[0], c) for c in rcols}
        with open(f"{prof}/{tag}_pmc_{cfg}.csv", "w") as f:
            cols = ["WRITE_SIZE_kB", *rcols] + (["FETCH_SIZE_kB"] if cfg == "b22" else [])
            f.write("dispatch," + ",".join(cols) + "\n")
            series = [write, *(rvals[c] for c in rcols)] + ([fetch] if cfg == "b22" else [])
            for i in range(max(len(v) for v in series)):
                f.write(f"{i}," + ",".join(str(v[i]) if i < len(v) else "" for v in series) + "\n")
        n = {c: med(rvals[c]) for c in rcols}
        # memory-side read requests by size: bytes = 32 n32 + 64 n64 + 128 n128 (requests of other
        # sizes, if any, are reported as the remainder and not counted); writes WRITE_SIZE (kB)
        read_bytes = 32 * n[rcols[1]] + 64 * n[rcols[2]] + 128 * n[rcols[3]]
        write_bytes = med(write) * 1024
        tc = {"batch": 65536, "kernel": kern[cfg],
              "rdreq": n, "rdreq_other": n[rcols[0]] - n[rcols[1]] - n[rcols[2]] - n[rcols[3]],
              "read_bytes": read_bytes, "write_bytes": write_bytes,
              "alg_bytes_per_launch": alg[cfg] * 65536,
              "hbm_bytes_per_launch": read_bytes + write_bytes,
              "ratio_to_algorithmic": (read_bytes + write_bytes) / (alg[cfg] * 65536),
              "dispatches": len(rvals[rcols[0]])}
        if cfg == "b22":
            tc["fetch_size_kB_raw"] = med(fetch)
            tc["read_bytes_fetch_size_x2"] = 2 * med(fetch) * 1024
        configs[cfg] = tc
    tj = {"source": f"profiles/{tag}_pmc_<config>.csv: medians over the dispatches after the first of one "
                    "rocprofv3 --pmc pass per counter group and config (bench.py --steps 5 --warmup 1); reads "
                    "from TCC_EA0_RDREQ_{32B,64B,128B}_sum (bytes by request size), writes WRITE_SIZE",
          "configs": configs}
    json.dump(tj, open(f"{prof}/pmc_traffic.json", "w"), indent=1)
    # this round's bench lines carry this round's traffic (bench.py read the previous
    # pmc_traffic.json when it ran, before these counter passes)
    for cfg, tc in configs.items():
        bp = f"{prof}/{tag}_bench_{cfg}.json"
        if os.path.exists(bp):
            bl = json.loads(open(bp).read())
            bl["roofline"]["traffic"] = tc["hbm_bytes_per_launch"]
            open(bp, "w").write(json.dumps(bl) + "\n")
    # agreement check: rocprofv3 kernel-trace durations of the timed dispatches vs the HIP-event
    # average bench.py measured in the same (profiled) process
    trace = one(f"{src}/trace/**/*kernel_trace.csv")
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            for r in csv.DictReader(open(trace)) if KERNEL in r["Kernel_Name"]]
    prof_line = [l for l in open(f"{src}/trace.log") if l.startswith("{")][-1]
    pb = json.loads(prof_line)
    steps, warm = pb["steps"], pb["warmup"]
    timed = durs[-steps:]  # the timed launches are the process's last `steps` dispatches (after settle + warmup)
    summary = {
        "kernel": configs["b22"]["kernel"],
        "rocprof_dispatches": len(durs),
        "rocprof_avg_ms_timed_dispatches": sum(timed) / len(timed),
        "bench_hip_event_avg_ms_same_process": pb["roofline"]["avg_kernel_ms"],
        "rel_diff": sum(timed) / len(timed) / pb["roofline"]["avg_kernel_ms"] - 1.0,
        "note": "trace run = python3 bench.py --steps %d --warmup %d under rocprofv3 --kernel-trace --stats" % (steps, warm),
    }
    json.dump(summary, open(f"{prof}/{tag}_trace_vs_bench.json", "w"), indent=1)
    print(json.dumps(summary, indent=1))
    print(json.dumps(tj, indent=1))
    print(open(f"{prof}/{tag}_kernel_stats.csv").read())


if __name__ == "__main__":
    main()

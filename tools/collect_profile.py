#!/usr/bin/env python3
"""Turns a tools/profile_round.sh output directory into the committed profile artefacts:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc.csv            per-dispatch FETCH_SIZE / WRITE_SIZE of the forward kernel
  profiles/pmc_traffic.json         HBM bytes per launch (read by bench.py for roofline.traffic)
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
    for cfg in ("b22", "c64", "d22"):
        p = f"{src}/bench_{cfg}.json"
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                open(f"{prof}/{tag}_bench_{cfg}.json", "w").write(lines[-1])
    fetch = pmc_values(one(f"{src}/pmc_fetch/**/*counter_collection.csv"), "FETCH_SIZE")
    write = pmc_values(one(f"{src}/pmc_write/**/*counter_collection.csv"), "WRITE_SIZE")
    rqf = glob.glob(f"{src}/pmc_rdreq/**/*counter_collection.csv", recursive=True)
    rcols = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
    rvals = {c: pmc_values(rqf[0], c) for c in rcols} if rqf else {c: [] for c in rcols}
    with open(f"{prof}/{tag}_pmc.csv", "w") as f:
        f.write("dispatch,FETCH_SIZE_kB,WRITE_SIZE_kB," + ",".join(rcols) + "\n")
        for i in range(max(len(fetch), len(write), *(len(v) for v in rvals.values()))):
            row = [fetch[i] if i < len(fetch) else "", write[i] if i < len(write) else ""]
            row += [rvals[c][i] if i < len(rvals[c]) else "" for c in rcols]
            f.write(f"{i}," + ",".join(str(x) for x in row) + "\n")
    # skip the first (warm-up) dispatch
    med = lambda v: sorted(v[1:] or v)[len(v[1:] or v) // 2]  # noqa: E731
    fk = med(fetch)
    wk = med(write)
    write_bytes = wk * 1024
    tj = {"config": "b22", "batch": 65536, "kernel": "k_forward<Cfg<22,1125,RB=1,CB=0>>",
          "fetch_size_kB_raw": fk, "write_size_kB": wk, "write_bytes": write_bytes,
          "alg_bytes_per_launch": (22 * 1125 + 4) * 65536}
    rq = glob.glob(f"{src}/pmc_rdreq/**/*counter_collection.csv", recursive=True)
    if rq:
        # memory-side read requests by size: bytes = 32 n32 + 64 n64 + 128 n128 (the requests of
        # other sizes, if any, are reported as the remainder and not counted)
        n = {c: med(pmc_values(rq[0], c)) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum",
                                                     "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")}
        read_bytes = 32 * n["TCC_EA0_RDREQ_32B_sum"] + 64 * n["TCC_EA0_RDREQ_64B_sum"] + 128 * n["TCC_EA0_RDREQ_128B_sum"]
        tj.update({"rdreq": n, "rdreq_other": n["TCC_EA0_RDREQ_sum"] - n["TCC_EA0_RDREQ_32B_sum"]
                   - n["TCC_EA0_RDREQ_64B_sum"] - n["TCC_EA0_RDREQ_128B_sum"],
                   "read_bytes": read_bytes, "read_bytes_fetch_size_x2": 2 * fk * 1024,
                   "source": f"profiles/{tag}_pmc.csv (medians over dispatches after the first); reads from "
                             "TCC_EA0_RDREQ_{32B,64B,128B}_sum (bytes by request size), writes WRITE_SIZE"})
    else:
        read_bytes = 2 * fk * 1024
        tj.update({"read_bytes": read_bytes,
                   "source": f"profiles/{tag}_pmc.csv (median over dispatches after the first; FETCH_SIZE x2 per gfx950 correction)"})
    tj["hbm_bytes_per_launch"] = read_bytes + write_bytes
    json.dump(tj, open(f"{prof}/pmc_traffic.json", "w"), indent=1)
    # the config-B bench line of this round carries this round's traffic (bench.py read the
    # previous pmc_traffic.json when it ran, before these counter passes)
    bp = f"{prof}/{tag}_bench_b22.json"
    if os.path.exists(bp):
        bl = json.loads(open(bp).read())
        bl["roofline"]["traffic"] = tj["hbm_bytes_per_launch"]
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
        "kernel": tj["kernel"],
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

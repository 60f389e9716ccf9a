#!/usr/bin/env python3
"""Targeted scan for the round-1 layer-1 fault's remaining candidate (candidate (ii)):
an MFMA whose C-init (srcC) registers were written by a VALU instruction at the compiler-minimum
distance while vector-memory loads into other registers are still outstanding (diagnostic).

For every MFMA with a VGPR srcC in the fused-kernel instantiations it walks back along the
straight-line code to the last instruction that wrote any srcC register and reports
  * the writer and its distance in wait states (instructions + s_nop counts),
  * how many vector-memory operations were outstanding when the writer issued (issue order, with
    every s_waitcnt vmcnt(N) applied; linear order, so a count across a branch is approximate),
  * or "loop-invariant" when no writer precedes it back to the loop head (the C-init is built
    once before the trial loop, where a full drain precedes the first layer 1).
A pattern hit is a writer within WINDOW wait states of the MFMA with at least one load outstanding.
Each MFMA is tagged with its barrier segment (s_barrier count before it): 0 the prologue, 1 layer 1
(up to barrier A), 2 layers 2-3, 3 layers 4-5.  tests/test_mfma_lint.py requires 0 hits in segment 1.

usage: python tools/cinit_scan.py mi-bminet_amd/build/mibminet.s [name-filter ...]
"""
import re
import sys

WINDOW = 4
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op):
    out = set()
    for m in REG.finditer(op):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def split_ops(rest):
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def parse(path):
    funcs, cur, name = {}, None, None
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name = m.group(1)
            cur = funcs.setdefault(name, [])
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        lab = re.match(r"^(\.LBB\S+):", line)
        if lab:
            cur.append(("label", lab.group(1), []))
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        parts = t.split(None, 1)
        cur.append((parts[0], t, split_ops(parts[1].split(";")[0]) if len(parts) > 1 else []))
    return funcs


def is_vmem(op):
    return op.startswith(("buffer_", "global_", "flat_", "scratch_"))


def writes(op, ops):
    """VGPRs the instruction writes (first operand of VALU, loads, DS reads)."""
    if not ops or op == "label":
        return set()
    if op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return regs(ops[0])
    if (is_vmem(op) and "load" in op and not op.endswith(" lds")) or (op.startswith("ds_read")):
        return regs(ops[0])
    return set()


def scan(funcs, filt):
    """Prints the report; returns the pattern hits as (function, segment, instruction)."""
    results = []
    for name, ins in funcs.items():
        if "k_forward" not in name or not all(f in name for f in filt):
            continue
        # outstanding vector-memory ops at each instruction (linear issue order)
        out, pend = [], 0
        for op, t, ops in ins:
            out.append(pend)
            if is_vmem(op):
                pend += 1
            m = re.search(r"vmcnt\((\d+)\)", t) if op == "s_waitcnt" else None
            if m:
                pend = min(pend, int(m.group(1)))
        short = re.sub(r"^_ZN3mib2wg9k_forwardINS0_3CfgI", "", name)[:40]
        hits, rows, seg = 0, [], 0
        for i, (op, t, ops) in enumerate(ins):
            if op == "s_barrier":
                seg += 1
            if not op.startswith("v_mfma") or len(ops) < 4 or not ops[3].startswith("v"):
                continue
            c = regs(ops[3])
            ws, j, found = 0, i - 1, None
            while j >= 0:
                oj, tj, opsj = ins[j]
                if oj == "label":
                    found = ("loop-invariant or across a branch", None)
                    break
                if writes(oj, opsj) & c:
                    # an earlier MFMA of the same chain: the accumulator itself, ordered by the
                    # hardware's MFMA dependency check, not a C-init
                    found = ("accumulation chain (MFMA)", None) if oj.startswith("v_mfma") else (tj, ws)
                    break
                ws += int(opsj[0]) + 1 if oj == "s_nop" else 1
                j -= 1
            if found is None or found[1] is None:
                rows.append(f"  seg {seg} {t[:60]:60s} srcC writer: {found[0] if found else 'none'}")
                continue
            wt, d = found
            hit = d <= WINDOW and out[j] > 0
            hits += hit
            if hit:
                results.append((name, seg, t))
            rows.append(f"  seg {seg} {t[:60]:60s} srcC writer {d} wait states before: {wt[:48]:48s} "
                        f"vmem outstanding {out[j]}{'   <-- pattern' if hit else ''}")
        print(f"{short}: {hits} pattern hit(s), {sum(1 for r in results if r[0] == name and r[1] == 1)} in layer 1")
        for r in rows:
            print(r)
    return results


if __name__ == "__main__":
    scan(parse(sys.argv[1]), sys.argv[2:])

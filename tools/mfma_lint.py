#!/usr/bin/env python3
"""Flags MFMA register patterns in device assembly that are suspect on gfx950 (diagnostic).

  partial dst/srcC overlap   vdst and srcC overlap without being identical
  dst partially over srcA/B  vdst overlaps a multiplicand of the same instruction without being it
  asm write into pending dst an inline-asm instruction (between ;;#ASMSTART and ;;#ASMEND) writes a
                             register of an earlier MFMA's destination that nothing has read yet:
                             the compiler's hazard checks do not see inline asm, and the MFMA's
                             write-back can land after the asm result (the round-2 layer-3 fault)

usage: python tools/mfma_lint.py mi-bminet_amd/build/mibminet.s
"""
import re
import sys


def rng(tok):
    tok = tok.strip().rstrip(",")
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return int(m.group(1)), int(m.group(2))
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return int(m.group(1)), int(m.group(1))
    return None


def ov(a, b):
    return a and b and not (a[1] < b[0] or b[1] < a[0])


def regs(tok):
    r = rng(tok)
    return set(range(r[0], r[1] + 1)) if r else set()


bad = 0
fn = None
lines = open(sys.argv[1]).read().split("\n")
# pass 1: inline-asm writes into MFMA destination registers that are still unread
in_asm = False
pending = {}  # reg -> line of the MFMA that writes it
for i, line in enumerate(lines):
    s = line.strip()
    if re.match(r"^_Z\S+:", s):
        fn = s.split(":")[0]
        pending = {}
    if s.startswith(";;#ASMSTART"):
        in_asm = True
        continue
    if s.startswith(";;#ASMEND"):
        in_asm = False
        continue
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        continue
    parts = s.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    srcs = set().union(*(regs(o.split()[0]) for o in ops[1:] if o)) if len(ops) > 1 else set()
    if op.startswith(("ds_write", "global_store", "buffer_store", "scratch_store")):
        srcs |= set().union(*(regs(o.split()[0]) for o in ops if o)) if ops else set()
        dst = set()
    else:
        dst = regs(ops[0].split()[0]) if ops and op.startswith(("v_", "ds_read", "global_load", "buffer_load")) else set()
    for r in srcs:
        pending.pop(r, None)
    if op.startswith("v_mfma"):
        for r in dst:
            pending[r] = i + 1
        continue
    hit = dst & set(pending)
    if hit and in_asm:
        bad += 1
        print(f"{i + 1}: {s}    <- asm write into pending dst of the MFMA at line {pending[min(hit)]}  [{fn[:60] if fn else '?'}]")
    for r in dst:
        pending.pop(r, None)
fn = None
for i, line in enumerate(lines):
    s = line.strip()
    if re.match(r"^_Z\S+:", s):
        fn = s.split(":")[0]
    if not s.startswith("v_mfma"):
        continue
    ops = [o.strip() for o in s.split(None, 1)[1].split(",")]
    d, a, b, c = (rng(o) for o in ops[:4])
    why = []
    if ov(d, c) and d != c:
        why.append("partial dst/srcC overlap")
    if (ov(d, a) and d != a) or (ov(d, b) and d != b):
        why.append("dst partially over srcA/srcB")
    if why:
        bad += 1
        print(f"{i + 1}: {s}    <- {', '.join(why)}  [{fn[:60] if fn else '?'}]")
print(f"{bad} suspect MFMA(s)")

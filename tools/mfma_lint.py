#!/usr/bin/env python3
"""Flags MFMA register patterns in device assembly that are suspect on gfx950 (diagnostic).

  partial dst/srcC overlap   vdst and srcC overlap without being identical
  dst partially over srcA/B  vdst overlaps a multiplicand of the same instruction without being it

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


bad = 0
fn = None
for i, line in enumerate(open(sys.argv[1])):
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

#!/usr/bin/env python3
"""Static instruction mix of the fused forward kernel, per barrier-delimited segment (and per basic
block inside each segment).  Usage: make -C mi-bminet_amd asm && python tools/isa_stats.py [cfg]"""
import re
import sys

cfg = sys.argv[1] if len(sys.argv) > 1 else "22ELi1125ELb1ELb0ELb0ELb0"
s = open("mi-bminet_amd/build/mibminet.s").read()
names = re.findall(r"^(_ZN3mib2wg9k_forward\S*):", s, re.M)
name = [n for n in names if cfg in n][0]
body = s[s.index(name + ":"):]
body = body[: body.index(".Lfunc_end")]


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "vmem"
    return "other"


seg, blk = 0, None
out = []
for raw in body.split("\n"):
    l = raw.strip()
    if not l or l.startswith(";") or (l.startswith(".") and not l.startswith(".LBB")):
        continue
    if l.startswith(".LBB"):
        blk = l.rstrip(":").split()[0]
        continue
    op = l.split()[0]
    out.append((seg, blk, op, l))
    if op == "s_barrier":
        seg += 1

from collections import Counter, OrderedDict
per = OrderedDict()
for sg, b, op, l in out:
    per.setdefault((sg, b), Counter())[cls(op)] += 1
for (sg, b), c in per.items():
    print(f"seg {sg:2d} {str(b):10s} " + " ".join(f"{k}={c[k]}" for k in ("valu", "mfma", "lds", "vmem", "salu", "wait")))
ops = Counter(op for _, _, op, _ in out if op.startswith("v_") and not op.startswith("v_mfma"))
print("top VALU ops:", ops.most_common(30))

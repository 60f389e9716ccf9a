#!/usr/bin/env python3
"""Compares the device assembly of two library builds kernel by kernel (diagnostic).

    python tools/asm_cmp.py before.s after.s      # each from `make -C mi-bminet_amd asm`

Kernels are matched by name; a Cfg<...> whose template list grew by trailing bool parameters
(e.g. Cfg::XR) is matched against the old name when the new parameters are all false.  Block
labels and comments are normalised, so "same" means the same instruction stream.
"""
import re
import sys


def norm(t):
    t = re.sub(r"\.LBB\d+_", ".LBB_", t)
    t = re.sub(r"\.Ltmp\d+", ".Ltmp", t)
    t = re.sub(r"\s*;.*", "", t)
    return "\n".join(line for line in t.splitlines() if line.strip())


def funcs(path):
    d, cur, buf = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if cur:
                d[cur] = norm("".join(buf))
            cur, buf = m.group(1), []
            continue
        if cur is not None:
            if line.startswith("\t.section") or line.startswith(".Lfunc_end"):
                d[cur], cur, buf = norm("".join(buf)), None, []
                continue
            buf.append(line)
    return d


def old_name(k, nold):
    m = re.search(r"CfgILi(\d+)ELi(\d+)((?:ELb[01])+)E", k)
    if not m:
        return k
    bools = re.findall(r"Lb([01])", m.group(3))
    if len(bools) <= nold:
        return k
    if any(b == "1" for b in bools[nold:]):
        return None
    return k.replace(m.group(0), "CfgILi%sELi%s%sE" % (m.group(1), m.group(2), "".join("ELb" + x for x in bools[:nold])))


def main():
    a, b = funcs(sys.argv[1]), funcs(sys.argv[2])
    nold = max((len(re.findall(r"Lb[01]", m.group(0))) for k in a for m in [re.search(r"CfgILi\d+ELi\d+(?:ELb[01])+E", k)] if m),
               default=0)
    bm = {}
    for k, v in b.items():
        o = old_name(k, nold)
        if o:
            bm[o] = v
    same = diff = 0
    for k in a:
        if k not in bm:
            print("missing", k)
        elif a[k] == bm[k]:
            same += 1
        else:
            diff += 1
            print("DIFF", k)
    print("same", same, "diff", diff, "new", len(b) - same - diff)
    return 1 if diff else 0


if __name__ == "__main__":
    sys.exit(main())

#!/bin/bash
# One line per k_forward instantiation: Cfg template args (C, T, RB, CB, CT, FQ, XR), VGPRs, scratch bytes/lane, LDS bytes.
# usage: tools/resource.sh [repo root]  (default: this checkout)
cd "${1:-$(dirname "$0")/..}/mi-bminet_amd"
make -s resource 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: _ZN3mib2wg9k_forwardINS0_3CfgILi(\d+)ELi(\d+)ELb(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)", line)
    if m:
        cur = "C=%s T=%s RB=%s CB=%s CT=%s FQ=%s XR=%s" % m.groups(); vals = {}
        continue
    if cur is None:
        continue
    for k in ("VGPRs", "ScratchSize [bytes/lane]", "LDS Size [bytes/block]"):
        m = re.search(re.escape(k) + r": (\d+)", line)
        if m:
            vals[k.split()[0]] = m.group(1)
    if len(vals) == 3:
        print(cur, " vgpr", vals["VGPRs"], " scratch", vals["ScratchSize"], " lds", vals["LDS"]); cur = None
'

"""Writer of the reference's generated parameter sources, net.h and net.c, from a ParamSet.

The reference turns a QuantLab export into C globals with ``edge-eegnet_wolf/data/gen_net_header.py``
(lines 49-224), formatted by ``python_utils/header_file.py``: ``#define`` constants for the
dimensions and the scalar factors, ``extern RT_L2_DATA const`` declarations in net.h and the
initialised arrays in net.c.  Its C layers read those globals directly (``src/cl/net/model.c``).
This writer produces the same names, types, layouts and file structure from the builder's own
``ParamSet`` (it never runs the reference), so that a C host can link a net.c exactly as the
reference's callers do and load it through ``net_params_load_arrays``
(``include/mibminet_net_h.h``), with no blob file and no Python at run time.

``runtime_include``: the header the generated net.h includes for the ``RT_L2_DATA`` placement
qualifier.  ``"rt/rt_api.h"`` (the PULP runtime) is what gen_net_header.py writes; ``None`` writes
an empty ``RT_L2_DATA`` definition instead, for hosts without the PULP runtime.
"""
from __future__ import annotations

import textwrap
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .params import ParamSet

WIDTH = 100   # header_file.py's line width
INDENT = "    "


def _comment(text: str) -> str:
    lines: List[str] = []
    for par in text.split("\n"):
        lines.extend(textwrap.wrap(par, WIDTH - 3) or [""])
    return "/*\n * " + "\n * ".join(lines) + "\n */\n\n"


def _array_def(name: str, ctype: str, data: Sequence[int]) -> str:
    values = ", ".join(str(int(v)) for v in data)
    one = f"RT_L2_DATA const {ctype} {name}[] = {{ {values} }};"
    if len(data) <= 16 and len(one) <= WIDTH:
        return one + "\n\n"
    body = textwrap.wrap(values, WIDTH - len(INDENT))
    return f"RT_L2_DATA const {ctype} {name}[] = {{\n" + INDENT + f"\n{INDENT}".join(body) + "};\n\n"


def net_h_sources(ps: ParamSet, runtime_include: Optional[str] = "rt/rt_api.h") -> Tuple[str, str]:
    """(net.h text, net.c text) holding ``ps`` as the reference's generated globals."""
    if ps.weight_bits != 8:
        raise ValueError("the reference's net.c holds int8 weights (weight_bits must be 8)")
    d = ps.dims
    T = d.T
    F2 = d.F2
    # (kind, name, value): kind "const" -> #define, "array" -> extern declaration + definition,
    # "comment" -> the layer banner
    entries: List[tuple] = [
        ("comment", "Network Dimensions", None),
        ("const", "NET_F1", d.F1), ("const", "NET_F2", F2), ("const", "NET_D", d.D),
        ("const", "NET_C", d.C), ("const", "NET_C_ALIGN", d.C_ALIGN), ("const", "NET_T", T),
        ("const", "NET_T_ALIGN", d.T_ALIGN), ("const", "NET_T8", d.T8), ("const", "NET_T8_ALIGN", d.T8_ALIGN),
        ("const", "NET_T64", d.T64), ("const", "NET_T64_ALIGN", d.T64_ALIGN), ("const", "NET_N", d.N),
        ("comment", "Layer 1\n=======\nConvolution + BN\n\nInput:  [C, T]\nWeight: [C, 1]\nOutput: [F2, 1, T]", None),
        ("array", ("net_l1_factor", "int32_t"), ps.l1_factor),
        ("array", ("net_l1_offset", "int32_t"), ps.l1_offset),
        ("const", "NET_L1_WEIGHT_LEN", d.C), ("const", "NET_L1_WEIGHT_LEN_ALIGN", d.C_ALIGN),
        ("array", ("net_l1_weight", "int8_t"), ps.w1()),
        ("array", ("net_l1_weight_align", "int8_t"), ps.l1_weight_align),
        ("array", ("net_l1_weight_32", "int32_t"), ps.w1()),
        ("comment", "Layer 2\n=======\nConvolution + BN + ReLU + Pooling\n\nInput:  [F2, 1, T]\n"
                    "Weight: [F2, 1, 64]\nOutput: [F2, T // 8]", None),
        ("const", "NET_L2_PAD_START", 31), ("const", "NET_L2_PAD_END", 32),
        ("const", "NET_L2_PAD_INPUT_LEN", T + 63), ("const", "NET_L2_PAD_INPUT_LEN_ALIGN", (T + 63 + 3) // 4 * 4),
        ("array", ("net_l2_factor", "int32_t"), ps.l2_factor),
        ("array", ("net_l2_offset", "int32_t"), ps.l2_offset),
        ("const", "NET_L2_WEIGHT_LEN", 64), ("const", "NET_L2_WEIGHT_LEN_ALIGN", 64),
        # conv order (flipped taps) and the cross-correlation order the canonical build reads
        ("array", ("net_l2_weight", "int8_t"), ps.l2_weight_reverse[:, ::-1]),
        ("array", ("net_l2_weight_reverse", "int8_t"), ps.l2_weight_reverse),
        ("array", ("net_l2_weight_reverse_pad", "int8_t"), ps.l2_weight_reverse),
        ("comment", "Layer 3\n=======\nConvolution\n\nInput:  [F2, T // 8]\nWeight: [F2, 16]\n"
                    "Output: [F2, T // 8]", None),
        ("const", "NET_L3_PAD_START", 7), ("const", "NET_L3_PAD_END", 8),
        ("const", "NET_L3_PAD_INPUT_LEN", d.T8 + 15), ("const", "NET_L3_PAD_INPUT_LEN_ALIGN", (d.T8 + 15 + 3) // 4 * 4),
        ("const", "NET_L3_FACTOR", ps.l3_factor), ("const", "NET_L3_WEIGHT_LEN", 16),
        ("array", ("net_l3_weight", "int8_t"), ps.l3_weight),
        ("comment", "Layer 4\n=======\nConvolution + BN + ReLU + Pooling\n\nInput:  [F2, T // 8]\n"
                    "Weight: [F2, F2]\nOutput: [F2, T // 64]", None),
        ("array", ("net_l4_factor", "int32_t"), ps.l4_factor),
        ("array", ("net_l4_offset", "int32_t"), ps.l4_offset),
        ("const", "NET_L4_WEIGHT_LEN", F2),
        ("array", ("net_l4_weight", "int8_t"), ps.l4_weight),
        ("comment", "Layer 5\n=======\nLinear Layer (without scaling in the end)\n\nInput:  [F2, T // 64]\n"
                    "Weight: [N, F2 * (T // 64)]\nBias:   [N]\nOutput: [N]", None),
        ("const", "NET_L5_FACTOR", ps.l5_factor),
        ("array", ("net_l5_bias", "int8_t"), ps.l5_bias),
        ("const", "NET_L5_WEIGHT_LEN", F2 * d.T64_ALIGN),
        ("array", ("net_l5_weight", "int8_t"), ps.l5_weight),
    ]
    guard = "__NET_NET_H__"
    h = [f"#ifndef {guard}\n#define {guard}\n\n"]
    if runtime_include:
        h.append(f'#include "{runtime_include}"\n\n')
    else:
        h.append("#include <stdint.h>\n\n#ifndef RT_L2_DATA\n#define RT_L2_DATA\n#endif\n\n")
    c = ['#include "net.h"\n\n']
    for kind, name, value in entries:
        if kind == "comment":
            text = "// " + name + "\n" if value is None and "\n" not in name else _comment(name)
            h.append(text)
            c.append(text if text.startswith("/*") else "")
        elif kind == "const":
            h.append(f"#define {name} {int(value)}\n")
        else:
            arr_name, ctype = name
            flat = np.asarray(value).ravel()
            h.append(f"extern RT_L2_DATA const {ctype} {arr_name}[{flat.size}];\n")
            c.append(_array_def(arr_name, ctype, flat))
    h.append(f"\n#endif//{guard}\n")
    return "".join(h), "".join(c)


def write_net_h(ps: ParamSet, directory: str, runtime_include: Optional[str] = "rt/rt_api.h") -> None:
    """Writes ``directory``/net.h and ``directory``/net.c."""
    import os

    h, c = net_h_sources(ps, runtime_include)
    with open(os.path.join(directory, "net.h"), "w") as f:
        f.write(h)
    with open(os.path.join(directory, "net.c"), "w") as f:
        f.write(c)

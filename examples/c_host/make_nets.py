"""Writes the generated weight sources the C host links (net_b22/, net_g19/): seeded synthetic
parameter sets in the reference's net.h / net.c format (mibminet/net_h.py), for hosts without the
PULP runtime (RT_L2_DATA defined empty).  tests/test_net_h.py regenerates them and compares."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "mi-bminet_amd"))

from mibminet.net_h import write_net_h  # noqa: E402
from mibminet.params import ParamSet  # noqa: E402

NETS = {
    "net_b22": dict(seed=22, C=22, T=1125, N=4),
    "net_g19": dict(seed=19, C=19, T=480, N=3),
}


def param_set(name):
    kw = dict(NETS[name])
    return ParamSet.synthetic(kw.pop("seed"), **kw)


def main(out=HERE):
    for name in NETS:
        d = os.path.join(out, name)
        os.makedirs(d, exist_ok=True)
        write_net_h(param_set(name), d, runtime_include=None)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else HERE)

"""mibminet — MI355X-native int8 inference path for the quantized MI-BMInet (edgeEEGNet).

* ``params``: the weight ABI (net.h arrays, blob format, QuantLab -> int parameter compiler).
* ``lib``: ctypes binding of libmibminet.so, the C ABI of include/mibminet.h (gfx950 HIP kernels);
  import it explicitly (``from mibminet import lib``).
"""
from .params import Dims, ParamSet, pack_trials, trial_stride_bytes  # noqa: F401

__all__ = ["Dims", "ParamSet", "pack_trials", "trial_stride_bytes"]

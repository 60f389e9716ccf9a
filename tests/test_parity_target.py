"""Which reference the results follow where the reference C and the golden model disagree
("Parity target").

The canonical C build (PARALLEL + REORDER_BN) writes each layer-2 filter row at stride NET_T8 in
the cluster's L1 buffer (layer2.c:78; the plain branch at :163), but the driver copies
NUM_WORKERS * NET_T8_ALIGN bytes per batch of filters back (layer2.c:313-315), and every reader
takes rows at stride NET_T8_ALIGN (layer3.c:131-135).  Layer 3's driver copies back only
NET_F2 * NET_T8 bytes of its [F2][T8_ALIGN] result image (layer3.c:153).  When T8 = T / 8 is a
multiple of 4 (config B: T8 = 140; 64 x 480: T8 = 60) both are exact.  Otherwise (config C,
T = 1000: T8 = 125, T8_ALIGN = 128) the rows the C hands on are shifted, the last row of each
batch ends in L1 bytes nobody wrote, and layer 3's last row keeps whatever the caller's buffer
held: the C's logits there depend on uninitialised memory, so they are no target.  The oracle (and
the GPU) follow python_utils/golden_model.py there, which has no such copy.  These tests restate
the C's copies on the oracle's own layer outputs and pin that choice."""
import numpy as np
import pytest

import oracle
from mibminet.params import ParamSet

NUM_WORKERS = 8  # rt_team_fork(NUM_WORKERS, ...) in layer2.c:311


def c_layer2_copy(y2, T8, fill):
    """The rows net_layer2 hands on in the C build: per batch of NUM_WORKERS filters, the kernel's
    rows at stride T8 (layer2.c:78) in an L1 buffer of NUM_WORKERS * T8_ALIGN bytes whose tail holds
    `fill` (rt_alloc'd, never written), copied out and read at stride T8_ALIGN."""
    F2, T8A = y2.shape
    out = np.zeros_like(y2)
    for b in range(F2 // NUM_WORKERS):
        loc = np.full(NUM_WORKERS * T8A, fill, np.int8)
        for w in range(NUM_WORKERS):
            loc[w * T8: (w + 1) * T8] = y2[b * NUM_WORKERS + w, :T8]
        out[b * NUM_WORKERS:(b + 1) * NUM_WORKERS] = loc.reshape(NUM_WORKERS, T8A)
    return out


def c_layer3_copy(y3, T8, caller_bytes):
    """net_layer3's copy-back (layer3.c:153): NET_F2 * NET_T8 bytes of the [F2][T8_ALIGN] image;
    the rest of the caller's buffer keeps `caller_bytes`."""
    F2, T8A = y3.shape
    out = np.asarray(caller_bytes, np.int8).reshape(F2 * T8A).copy()
    out[: F2 * T8] = y3.ravel()[: F2 * T8]
    return out.reshape(F2, T8A)


def c_model(co, x, T8, fill):
    """The C build's forward with its copies restated (layers from the oracle)."""
    y1 = co.layer1(x)
    y2 = c_layer2_copy(co.layer2(y1), T8, fill)
    y3 = c_layer3_copy(co.layer3(y2), T8, np.full(y2.size, fill, np.int8))
    return co.layer5(co.layer4(co.layer3_flip(y3)))


@pytest.mark.parametrize("C,T", [(22, 1125), (64, 480), (8, 512)])
def test_c_copies_are_exact_when_t8_is_aligned(C, T):
    """T8 % 4 == 0: the C's copies change nothing, so the C, the golden model and the oracle agree."""
    ps = ParamSet.synthetic(seed=T, C=C, T=T)
    d = ps.dims
    assert d.T8 % 4 == 0
    co = oracle.COracle(ps)
    rng = np.random.default_rng(C)
    for _ in range(3):
        x = oracle.to_tc_align(rng.integers(-128, 128, size=(C, T)), d.C_ALIGN)
        y2 = co.layer2(co.layer1(x))
        for fill in (0, 85, -86):
            np.testing.assert_array_equal(c_layer2_copy(y2, d.T8, fill), y2)
            np.testing.assert_array_equal(c_model(co, x, d.T8, fill), co.model(x))


def test_c_copies_shift_rows_when_t8_is_not_aligned():
    """Config C (T = 1000, T8 = 125): the C's layer-2 rows are shifted and its logits depend on the
    contents of memory it never wrote; the oracle (= the golden model, checked in
    tests/test_oracle.py) is the deterministic target."""
    ps = ParamSet.synthetic(seed=1000, C=64, T=1000)
    d = ps.dims
    assert (d.T8, d.T8_ALIGN) == (125, 128)
    co = oracle.COracle(ps)
    rng = np.random.default_rng(64)
    differ, fill_dependent = 0, 0
    for _ in range(8):
        x = oracle.to_tc_align(rng.integers(-128, 128, size=(64, 1000)), d.C_ALIGN)
        y2 = co.layer2(co.layer1(x))
        c2 = c_layer2_copy(y2, d.T8, 0)
        # filter 0 of each batch is intact; filter w starts 3 w elements late
        np.testing.assert_array_equal(c2[0, :125], y2[0, :125])
        np.testing.assert_array_equal(c2[1, :122], y2[1, 3:125])
        assert not np.array_equal(c2[:, :125], y2[:, :125])
        logits = [c_model(co, x, d.T8, fill) for fill in (0, 127, -128)]
        differ += not np.array_equal(logits[0], co.model(x))
        fill_dependent += not (np.array_equal(logits[0], logits[1]) and np.array_equal(logits[1], logits[2]))
    assert differ >= 6       # the shifted rows change the logits
    assert fill_dependent >= 1  # and the C's own result is not a function of its inputs

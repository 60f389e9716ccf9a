"""Parameter blob (weight ABI) round trips and validation — host logic, CPU only."""
import numpy as np
import pytest

from mibminet.params import ParamSet, appendix_b_net, pack_trials, trial_stride_bytes, _pack_int4, _unpack_int4


@pytest.mark.parametrize("C,T,wbits", [(22, 1125, 8), (64, 1000, 8), (22, 1125, 4), (22, 1125, 4)])
def test_blob_roundtrip(C, T, wbits):
    ps = ParamSet.synthetic(seed=3, C=C, T=T, weight_bits=wbits)
    blob = ps.to_blob()
    assert len(blob) % 4 == 0
    q = ParamSet.from_blob(blob)
    assert q.dims == ps.dims and q.weight_bits == wbits
    for name in ("l1_factor", "l1_offset", "l1_weight_align", "l2_factor", "l2_offset", "l2_weight_reverse",
                 "l3_weight", "l4_factor", "l4_offset", "l4_weight", "l5_bias", "l5_weight"):
        assert np.array_equal(getattr(q, name), getattr(ps, name)), name
    assert q.l3_factor == ps.l3_factor and q.l5_factor == ps.l5_factor
    assert q.to_blob() == blob


def test_int4_packing():
    a = np.arange(-8, 8, dtype=np.int8)
    assert np.array_equal(_unpack_int4(_pack_int4(a), a.size), a)
    odd = np.array([-8, 7, 3], np.int8)
    assert np.array_equal(_unpack_int4(_pack_int4(odd), 3), odd)
    # nibble order: element 0 in the low nibble
    assert _pack_int4(np.array([1, -1], np.int8)) == bytes([0xF1])
    with pytest.raises(ValueError):
        _pack_int4(np.array([9], np.int8))


def test_int4_blob_is_smaller():
    p8 = ParamSet.synthetic(seed=1, weight_bits=8)
    p4 = ParamSet.synthetic(seed=1, weight_bits=4)
    assert len(p4.to_blob()) < len(p8.to_blob())


def test_validation():
    ps = ParamSet.synthetic(seed=2)
    blob = bytearray(ps.to_blob())
    with pytest.raises(ValueError):
        ParamSet.from_blob(bytes(blob[:-4]))
    bad = bytearray(blob)
    bad[0:8] = b"NOTMIBMI"
    with pytest.raises(ValueError):
        ParamSet.from_blob(bytes(bad))
    with pytest.raises(ValueError):
        ParamSet(ps.dims, np.zeros(16), ps.l1_offset, ps.l1_weight_align, ps.l2_factor, ps.l2_offset,
                 ps.l2_weight_reverse, ps.l3_factor, ps.l3_weight, ps.l4_factor, ps.l4_offset,
                 ps.l4_weight, ps.l5_factor, ps.l5_bias, ps.l5_weight)
    w = ps.l1_weight_align.copy()
    w[0, 23] = 1  # padding must be zero (gen_net_header.py align_array)
    with pytest.raises(ValueError):
        ParamSet(ps.dims, ps.l1_factor, ps.l1_offset, w, ps.l2_factor, ps.l2_offset,
                 ps.l2_weight_reverse, ps.l3_factor, ps.l3_weight, ps.l4_factor, ps.l4_offset,
                 ps.l4_weight, ps.l5_factor, ps.l5_bias, ps.l5_weight)


def test_quantlab_layouts():
    """net.h layout conventions of gen_net_header: l1/l2 stored in torch order, l3 flipped."""
    net, cfg, _ = appendix_b_net(0)
    ps = ParamSet.from_quantlab(net, cfg)
    from mibminet.params import quantize_to_int
    w2 = quantize_to_int(net["conv2.weightFrozen"], net["conv2.sParam"][0]).reshape(16, 64)
    assert np.array_equal(ps.l2_weight_reverse, w2)
    w3 = quantize_to_int(net["sep_conv1.weightFrozen"], net["sep_conv1.sParam"][0]).reshape(16, 16)
    assert np.array_equal(ps.l3_weight, w3[:, ::-1])
    assert np.all(ps.l1_weight_align[:, 22:] == 0)
    w5 = ps.l5_weight.reshape(4, 16, 20)
    assert np.all(w5[:, :, 17:] == 0)


def test_pack_trials_layout():
    x = np.arange(2 * 3 * 70).reshape(2, 3, 70) % 100
    p = pack_trials(x)
    assert p.shape == (2, trial_stride_bytes(3, 70)) and p.shape[1] % 16 == 0
    assert p[1, 5 * 3 + 2] == x[1, 2, 5]
    assert np.all(p[:, 210:] == 0)

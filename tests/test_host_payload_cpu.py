"""Host-only helpers of the C ABI on payload bytes (no device needed): skml_dense_info_host,
skml_dense_bins_host and skml_dense_times_by_host over a payload laid out by hand from the
oracle's QuantileQuantizer result (include/skml.h: 64-byte header, double splits padded to 256
bytes, LSB-first packed codes)."""
import ctypes as C
import struct

import numpy as np
import pytest

from oracle import oracle as O


def _payload(oq, n, req_bins):
    bits = 1
    while (1 << bits) < oq.bin_num:
        bits <<= 1
    off = (64 + 8 * (req_bins - 1) + 255) // 256 * 256
    hdr = struct.pack("<Iiqiiiiddqq", 0x444D4B53, 0, n, oq.bin_num, oq.zero_idx, bits, req_bins, oq.min, oq.max, off, 0)
    body = bytearray(off + (n * bits + 7) // 8)
    body[:64] = hdr
    body[64:64 + 8 * (oq.bin_num - 1)] = oq.splits.astype("<f8").tobytes()
    if bits == 16:
        body[off:] = oq.bins.astype("<u2").tobytes()
    else:
        per = 8 // bits
        b = oq.bins.astype(np.uint32)
        pad = (-len(b)) % per
        b = np.concatenate([b, np.zeros(pad, np.uint32)]).reshape(-1, per)
        packed = np.zeros(len(b), np.uint32)
        for k in range(per):
            packed |= b[:, k] << (k * bits)
        body[off:] = packed.astype(np.uint8).tobytes()
    return np.frombuffer(bytes(body), dtype=np.uint8).copy()


@pytest.mark.parametrize("n,bins", [(1000, 256), (70001, 4), (5000, 1000), (33333, 2), (4099, 16)])
def test_host_payload_helpers(n, bins):
    from sketchml_amd import _lib as L
    x = np.random.default_rng(n).standard_normal(n)
    oq = O.quantize(x, bins, 5)
    pl = _payload(oq, n, bins)
    h = L.DenseHeader()
    sp = np.zeros(bins, dtype=np.float64)
    assert L.lib.skml_dense_info_host(pl.ctypes.data_as(C.c_void_p), len(pl), C.byref(h), sp.ctypes.data_as(L.dblp),
                                      bins) == 0
    assert (h.bin_num, h.zero_idx, h.n) == (oq.bin_num, oq.zero_idx, n)
    assert np.array_equal(sp[: oq.bin_num - 1], oq.splits)
    got = np.zeros(n, dtype=np.int32)
    assert L.lib.skml_dense_bins_host(pl.ctypes.data_as(C.c_void_p), len(pl), got.ctypes.data_as(C.c_void_p), n) == 0
    assert np.array_equal(got, oq.bins)
    assert L.lib.skml_dense_times_by_host(pl.ctypes.data_as(C.c_void_p), len(pl), -3.0) == 0
    O.lib().orc_times_by(C.byref(oq.hdr), -3.0)
    assert L.lib.skml_dense_info_host(pl.ctypes.data_as(C.c_void_p), len(pl), C.byref(h), sp.ctypes.data_as(L.dblp),
                                      bins) == 0
    assert (h.min, h.max) == (oq.hdr.min, oq.hdr.max)
    assert np.array_equal(sp[: oq.bin_num - 1], np.array(oq.hdr.splits[: oq.bin_num - 1]))


def test_host_payload_rejects_malformed():
    from sketchml_amd import _lib as L
    x = np.random.default_rng(1).standard_normal(100)
    oq = O.quantize(x, 8, 1)
    pl = _payload(oq, 100, 8)
    bins = np.zeros(100, dtype=np.int32)
    ptr = pl.ctypes.data_as(C.c_void_p)
    assert L.lib.skml_dense_bins_host(ptr, len(pl) - 1, bins.ctypes.data_as(C.c_void_p), 100) == L.SKML_E_ARG
    assert L.lib.skml_dense_bins_host(ptr, len(pl), bins.ctypes.data_as(C.c_void_p), 99) == L.SKML_E_ARG
    bad = pl.copy()
    bad[0] ^= 1  # magic
    assert L.lib.skml_dense_bins_host(bad.ctypes.data_as(C.c_void_p), len(bad), bins.ctypes.data_as(C.c_void_p),
                                      100) == L.SKML_E_STATE
    for off, val in ((24, 7), (20, 8), (23, 0x80)):  # code_bits vs bin_num; zeroIdx == binNum; zeroIdx < 0
        bad = pl.copy()
        bad[off] = val
        assert L.lib.skml_dense_bins_host(bad.ctypes.data_as(C.c_void_p), len(bad), bins.ctypes.data_as(C.c_void_p),
                                          100) == L.SKML_E_ARG

"""Host-memory entry points (the JNI path: a JVM float[] in, payload bytes out, and back):
skml_dense_encode_host_f32 / skml_dense_decode_host_f32, from pageable numpy memory (staged
through the library's pinned pair) and from pinned memory (skml_host_alloc, the Java direct
ByteBuffer case).  The payload equals the device-resident encode byte for byte, the bins and
splits equal the oracle's."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _L():
    from sketchml_amd import _lib
    return _lib


def _params(bins=256, seed=0):
    L = _L()
    p = L.Params()
    L.lib.skml_params_default(C.byref(p))
    p.bin_num, p.seed = bins, seed
    return p


def _encode_host(gpu, x, bins, seed):
    L = _L()
    ctx = gpu.get_context()
    cap = C.c_size_t()
    assert L.lib.skml_dense_encode_host_f32(ctx.handle, None, len(x), C.byref(_params(bins, seed)), None, 0,
                                            C.byref(cap)) == 0
    out = np.zeros(cap.value, dtype=np.uint8)
    wrote = C.c_size_t()
    st = L.lib.skml_dense_encode_host_f32(ctx.handle, x.ctypes.data_as(C.c_void_p), len(x),
                                          C.byref(_params(bins, seed)), out.ctypes.data_as(C.c_void_p),
                                          out.nbytes, C.byref(wrote))
    return st, out[: wrote.value]


def _device_payload(gpu, x, bins, seed, nbytes):
    L = _L()
    ctx = gpu.get_context()
    xd = torch.from_numpy(x).cuda()
    nb = L.lib.skml_dense_payload_bytes(len(x), bins)
    pl = gpu.alloc_aligned(nb, "cuda")
    assert L.lib.skml_dense_encode_f32(ctx.handle, C.c_void_p(xd.data_ptr()), len(x), C.byref(_params(bins, seed)),
                                       C.c_void_p(pl.data_ptr()), nb) == 0
    torch.cuda.synchronize()
    return pl[:nbytes].cpu().numpy()


def _check_payload(pl, x, bins, seed):
    L = _L()
    h = L.DenseHeader.from_buffer_copy(pl[:64].tobytes())
    oq = O.quantize(x.astype(np.float64), bins, seed)
    assert (h.magic, h.n, h.bin_num, h.zero_idx, h.min, h.max) == (
        0x444D4B53, len(x), oq.bin_num, oq.zero_idx, oq.min, oq.max)
    sp = np.frombuffer(pl[64: 64 + 8 * (oq.bin_num - 1)].tobytes(), dtype=np.float64)
    assert np.array_equal(sp, oq.splits)
    return h, oq


@pytest.mark.parametrize("n", [1, 1000, 2**20 + 12345, 3 * 2**22 + 5])  # 1 piece .. several 8 MiB pieces
def test_encode_host_pageable_matches_device_and_oracle(gpu, n):
    x = np.random.default_rng(n).standard_normal(n, dtype=np.float32)
    st, pl = _encode_host(gpu, x, 256, 9)
    assert st == 0, _L().last_error()
    h, oq = _check_payload(pl, x, 256, 9)
    assert len(pl) == h.codes_offset + (n * h.code_bits + 7) // 8
    dev = _device_payload(gpu, x, 256, 9, len(pl))
    assert np.array_equal(pl, dev)
    # back: decode from the host payload into a host float[]
    out = np.zeros(n, dtype=np.float32)
    L = _L()
    assert L.lib.skml_dense_decode_host_f32(gpu.get_context().handle, pl.ctypes.data_as(C.c_void_p), len(pl),
                                            out.ctypes.data_as(C.c_void_p), n) == 0
    assert np.array_equal(out, oq.values()[oq.bins].astype(np.float32))


def test_encode_host_pinned_buffers(gpu):
    """Input and output in skml_host_alloc memory (DMA straight from / to them)."""
    L = _L()
    n = 2**22 + 77
    src = np.random.default_rng(3).standard_normal(n, dtype=np.float32)
    px, pp = C.c_void_p(), C.c_void_p()
    cap = L.lib.skml_dense_payload_bytes(n, 256)
    assert L.lib.skml_host_alloc(4 * n, C.byref(px)) == 0
    assert L.lib.skml_host_alloc(cap, C.byref(pp)) == 0
    try:
        xv = np.ctypeslib.as_array(C.cast(px, C.POINTER(C.c_float)), shape=(n,))
        xv[:] = src
        wrote = C.c_size_t()
        ctx = gpu.get_context()
        assert L.lib.skml_dense_encode_host_f32(ctx.handle, px, n, C.byref(_params(256, 4)), pp, cap,
                                                C.byref(wrote)) == 0, L.last_error()
        pl = np.ctypeslib.as_array(C.cast(pp, C.POINTER(C.c_uint8)), shape=(wrote.value,)).copy()
        _check_payload(pl, src, 256, 4)
        assert np.array_equal(pl, _device_payload(gpu, src, 256, 4, len(pl)))
    finally:
        L.lib.skml_host_free(px)
        L.lib.skml_host_free(pp)


def test_encode_host_errors(gpu):
    L = _L()
    x = np.random.default_rng(1).standard_normal(5000, dtype=np.float32)
    x[10] = np.nan
    st, _ = _encode_host(gpu, x, 256, 1)
    assert st == L.SKML_E_NAN
    x[10] = 0.0
    out = np.zeros(100, dtype=np.uint8)
    wrote = C.c_size_t()
    st = L.lib.skml_dense_encode_host_f32(gpu.get_context().handle, x.ctypes.data_as(C.c_void_p), len(x),
                                          C.byref(_params(256, 1)), out.ctypes.data_as(C.c_void_p), out.nbytes,
                                          C.byref(wrote))
    assert st == L.SKML_E_ARG and wrote.value > 100  # capacity too small, the needed size reported
    st, pl = _encode_host(gpu, x, 256, 1)
    assert st == 0
    dec = np.zeros(len(x), dtype=np.float32)
    assert L.lib.skml_dense_decode_host_f32(gpu.get_context().handle, pl.ctypes.data_as(C.c_void_p), len(pl) - 1,
                                            dec.ctypes.data_as(C.c_void_p), len(x)) == L.SKML_E_ARG  # truncated
    assert L.lib.skml_dense_decode_host_f32(gpu.get_context().handle, pl.ctypes.data_as(C.c_void_p), len(pl),
                                            dec.ctypes.data_as(C.c_void_p), len(x) + 1) == L.SKML_E_ARG  # wrong n


def test_encode_host_f64_and_host_helpers(gpu):
    """The double[] entry (the reference's own input), getBins / info / timesBy on the host
    payload, and decode back into a double[]."""
    L = _L()
    ctx = gpu.get_context()
    n = 2**20 + 333
    x = np.random.default_rng(8).standard_normal(n)  # float64
    cap = C.c_size_t()
    assert L.lib.skml_dense_encode_host_f64(ctx.handle, None, n, C.byref(_params(300, 2)), None, 0, C.byref(cap)) == 0
    pl = np.zeros(cap.value, dtype=np.uint8)
    wrote = C.c_size_t()
    assert L.lib.skml_dense_encode_host_f64(ctx.handle, x.ctypes.data_as(C.c_void_p), n, C.byref(_params(300, 2)),
                                            pl.ctypes.data_as(C.c_void_p), pl.nbytes, C.byref(wrote)) == 0
    pl = pl[: wrote.value]
    oq = O.quantize(x, 300, 2)
    h = L.DenseHeader()
    sp = np.zeros(400, dtype=np.float64)
    assert L.lib.skml_dense_info_host(pl.ctypes.data_as(C.c_void_p), len(pl), C.byref(h),
                                      sp.ctypes.data_as(L.dblp), 400) == 0
    assert (h.bin_num, h.zero_idx, h.min, h.max, h.n) == (oq.bin_num, oq.zero_idx, oq.min, oq.max, n)
    assert np.array_equal(sp[: h.bin_num - 1], oq.splits)
    bins = np.zeros(n, dtype=np.int32)
    assert L.lib.skml_dense_bins_host(pl.ctypes.data_as(C.c_void_p), len(pl), bins.ctypes.data_as(C.c_void_p), n) == 0
    assert np.array_equal(bins, oq.bins)
    assert L.lib.skml_dense_times_by_host(pl.ctypes.data_as(C.c_void_p), len(pl), 0.5) == 0
    O.lib().orc_times_by(C.byref(oq.hdr), 0.5)
    want = O.OracleQuant(oq.hdr, oq.bins).values()[oq.bins]
    out = np.zeros(n, dtype=np.float64)
    assert L.lib.skml_dense_decode_host_f64(ctx.handle, pl.ctypes.data_as(C.c_void_p), len(pl),
                                            out.ctypes.data_as(C.c_void_p), n) == 0
    assert np.array_equal(out, want)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_encode_host_uniform_quant_type(gpu, dtype):
    """params.quant_type = SKML_UNIFORM on the host entry points (the JNI encodeDenseUniformF64 /
    HipUniformQuantizer path): UniformQuantizer.quantize (quantization/UniformQuantizer.java:21-45)
    against the oracle, and byte-equal to the device-resident skml_dense_encode_uniform_*."""
    L = _L()
    ctx = gpu.get_context()
    n = 2**20 + 4321
    x = np.random.default_rng(12).standard_normal(n)
    if dtype == "f32":
        x = x.astype(np.float32)
    p = _params(256, 0)
    p.quant_type = L.SKML_UNIFORM
    enc_host = L.lib.skml_dense_encode_host_f32 if dtype == "f32" else L.lib.skml_dense_encode_host_f64
    cap = C.c_size_t()
    assert enc_host(ctx.handle, None, n, C.byref(p), None, 0, C.byref(cap)) == 0
    pl = np.zeros(cap.value, dtype=np.uint8)
    wrote = C.c_size_t()
    assert enc_host(ctx.handle, x.ctypes.data_as(C.c_void_p), n, C.byref(p), pl.ctypes.data_as(C.c_void_p),
                    pl.nbytes, C.byref(wrote)) == 0, L.last_error()
    pl = pl[: wrote.value]
    oq = O.uniform_quantize(x.astype(np.float64), 256)
    h = L.DenseHeader()
    sp = np.zeros(256, dtype=np.float64)
    assert L.lib.skml_dense_info_host(pl.ctypes.data_as(C.c_void_p), len(pl), C.byref(h),
                                      sp.ctypes.data_as(L.dblp), 256) == 0
    assert (h.bin_num, h.zero_idx, h.min, h.max, h.n) == (oq.bin_num, oq.zero_idx, oq.min, oq.max, n)
    assert np.array_equal(sp[: h.bin_num - 1], oq.splits)
    bins = np.zeros(n, dtype=np.int32)
    assert L.lib.skml_dense_bins_host(pl.ctypes.data_as(C.c_void_p), len(pl), bins.ctypes.data_as(C.c_void_p), n) == 0
    assert np.array_equal(bins, oq.bins)
    xd = torch.from_numpy(x).cuda()
    nb = L.lib.skml_dense_payload_bytes(n, 256)
    dpl = gpu.alloc_aligned(nb, "cuda")
    enc_dev = L.lib.skml_dense_encode_uniform_f32 if dtype == "f32" else L.lib.skml_dense_encode_uniform_f64
    assert enc_dev(ctx.handle, C.c_void_p(xd.data_ptr()), n, C.byref(p), C.c_void_p(dpl.data_ptr()), nb) == 0
    torch.cuda.synchronize()
    assert np.array_equal(pl, dpl[: len(pl)].cpu().numpy())


def test_sparse_and_delta_host_entries(gpu):
    L = _L()
    ctx = gpu.get_context()
    rng = np.random.default_rng(5)
    keys = np.nonzero(rng.random(400000) < 0.1)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys)).astype(np.float32)
    p = _params(256, 3)
    p.hash_seed = 4
    h = C.c_void_p()
    assert L.lib.skml_sparse_encode_kv_host_f32(ctx.handle, keys.ctypes.data_as(C.c_void_p),
                                                vals.ctypes.data_as(C.c_void_p), len(keys), C.byref(p),
                                                C.byref(h)) == 0, L.last_error()
    try:
        rk = np.zeros(len(keys), dtype=np.int32)
        rv = np.zeros(len(keys), dtype=np.float32)
        assert L.lib.skml_sparse_decode_host_f32(ctx.handle, h, rk.ctypes.data_as(C.c_void_p),
                                                 rv.ctypes.data_as(C.c_void_p)) == 0
    finally:
        L.lib.skml_sparse_free(h)
    osp = O.sparse_compress(keys, vals.astype(np.float64), 256, 8, 2, 0.3, 3, 4)
    ok, ob = osp.restore()
    assert np.array_equal(rk, ok)
    assert np.array_equal(rv, osp.q.values()[ob].astype(np.float32))
    # DeltaAdaptiveEncoder as a BinaryEncoder over host int[] / long[]
    ref = O.delta_encode(keys)
    m, kind = C.c_int32(), C.c_int32()
    nfb, ndb = C.c_int64(), C.c_int64()
    cap = len(keys)
    fw = np.zeros(cap, dtype=np.uint64)
    dw = np.zeros(cap, dtype=np.uint64)
    assert L.lib.skml_delta_encode_host(ctx.handle, keys.ctypes.data_as(C.c_void_p), len(keys), C.byref(m),
                                        C.byref(kind), C.byref(nfb), C.byref(ndb), fw.ctypes.data_as(C.c_void_p),
                                        dw.ctypes.data_as(C.c_void_p), cap) == 0, L.last_error()
    assert (m.value, bool(kind.value), nfb.value, ndb.value) == (
        ref["num_intervals"], ref["flag_kind"], ref["n_flag_bits"], ref["n_delta_bits"])
    nf, nd = len(ref["flag_words"]), len(ref["delta_words"])
    assert np.array_equal(fw[:nf], ref["flag_words"]) and np.array_equal(dw[:nd], ref["delta_words"])
    back = np.zeros(len(keys), dtype=np.int32)
    assert L.lib.skml_delta_decode_host(ctx.handle, len(keys), m.value, kind.value, ref["flag_words"].ctypes.data_as(C.c_void_p),
                                        nf, ref["delta_words"].ctypes.data_as(C.c_void_p), nd,
                                        back.ctypes.data_as(C.c_void_p)) == 0, L.last_error()
    assert np.array_equal(back, keys)

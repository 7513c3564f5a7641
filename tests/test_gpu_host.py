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

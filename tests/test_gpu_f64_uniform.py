"""GPU parity of the fp64-input quantile path and the uniform quantizer
against the CPU restatement.

fp64 quantile (QuantileQuantizer.quantize(double[]), QuantileQuantizer.java:27-50): the same bar
as the fp32 path -- same seed -> bin_num, zero_idx, min, max and splits equal, bins bit-exact,
decoded doubles bit-exact to the oracle's getValues()[bin].

Uniform (UniformQuantizer.java:21-45), fp32 and fp64 input: header, splits (sequential `+=`
accumulation) and bins bit-exact, including NaN values (binned by indexOf), the Double.MIN_VALUE
max quirk, the first-zero-wins min, and degenerate ranges whose split tables are NaN or +inf.
All device work goes through libskml.so; the oracle is only the checker.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _data64(n, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        return rng.standard_normal(n)
    if kind == "app":
        return np.where(rng.random(n) < 0.9, rng.standard_normal(n), 0.0)
    if kind == "signed_zero":
        x = rng.standard_normal(n)
        r = rng.random(n)
        x[r < 0.2] = 0.0
        x[(r >= 0.2) & (r < 0.4)] = -0.0
        return x
    if kind == "dups":
        return rng.integers(-5, 6, n).astype(np.float64)
    if kind == "special":
        x = rng.standard_normal(n) * 1e200
        x[rng.random(n) < 0.05] = 1e-310   # fp64 denormal
        x[rng.random(n) < 0.05] = -1e-310
        x[rng.random(n) < 0.01] = np.inf
        x[rng.random(n) < 0.01] = -np.inf
        return x
    if kind == "close":  # values that differ only below fp32 precision
        return 1.0 + rng.integers(0, 1000, n) * 2.0**-40
    if kind == "negative":
        return -np.abs(rng.standard_normal(n)) - 0.5
    if kind == "const":
        return np.full(n, 3.25)
    raise ValueError(kind)


def _check(gq, oq, x):
    assert gq.getBinNum() == oq.bin_num
    assert gq.getZeroIdx() == oq.zero_idx
    assert np.float64(gq.getMin()).tobytes() == np.float64(oq.min).tobytes()
    assert np.float64(gq.getMax()).tobytes() == np.float64(oq.max).tobytes()
    gs = gq.getSplits()
    assert gs.shape == oq.splits.shape
    assert np.array_equal(gs, oq.splits, equal_nan=True)
    gb = gq.getBins().cpu().numpy()
    assert np.array_equal(gb, oq.bins)


SIZES64 = [1, 100, 255, 256, 257, 1000, 16384, 16384 + 300, 65536, 65536 * 2 + 777, 2**20 + 12345]


@pytest.mark.parametrize("n", SIZES64)
def test_f64_quantize_matches_oracle(gpu, n):
    x = _data64(n, n + 1)
    gq = gpu.QuantileQuantizer(256, seed=n % 97)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.quantize(x, 256, n % 97)
    _check(gq, oq, x)
    dec = gq.decode()
    assert dec.dtype == torch.float64
    assert np.array_equal(dec.cpu().numpy(), oq.values()[oq.bins])


@pytest.mark.parametrize("kind", ["app", "signed_zero", "dups", "special", "close", "negative", "const"])
@pytest.mark.parametrize("n", [300, 4096 * 3 + 11, 2**17 + 5])
def test_f64_edge_data(gpu, kind, n):
    x = _data64(n, 7, kind)
    gq = gpu.QuantileQuantizer(256, seed=31)
    gq.quantize(torch.from_numpy(x).cuda())
    _check(gq, O.quantize(x, 256, 31), x)


def test_f64_large_pow2(gpu):
    n = 2**22
    x = _data64(n, 3)
    gq = gpu.QuantileQuantizer(256, seed=12)
    gq.quantize(torch.from_numpy(x).cuda())
    _check(gq, O.quantize(x, 256, 12), x)


@pytest.mark.timeout(300)
def test_f64_bench_workload_2p26_matches_oracle(gpu):
    """bench.py's extras.other_configs.fp64_encode workload at its timed size: 2^26 doubles drawn on
    the device by torch.randn(float64) under generator seed 4, 256 requested bins, the default
    params (seed 0).  Header, splits, every bin and every decoded double against the oracle's
    QuantileQuantizer.quantize(double[]) (QuantileQuantizer.java:27-50) over the same values."""
    import ctypes as C
    from sketchml_amd import _lib as L
    ctx = gpu.get_context()
    n = 2**26
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    p = L.Params()
    L.lib.skml_params_default(C.byref(p))
    p.bin_num = 256
    nb = L.lib.skml_dense_payload_bytes(n, 256)
    pl = gpu.alloc_aligned(nb, "cuda")
    assert L.lib.skml_dense_encode_f64(ctx.handle, C.c_void_p(x.data_ptr()), n, C.byref(p),
                                       C.c_void_p(pl.data_ptr()), nb) == 0, L.last_error()
    dec = torch.empty(n, dtype=torch.float64, device="cuda")
    assert L.lib.skml_dense_decode_f64(ctx.handle, C.c_void_p(pl.data_ptr()), C.c_void_p(dec.data_ptr()), n) == 0
    bins = torch.empty(n, dtype=torch.int32, device="cuda")
    assert L.lib.skml_dense_bins_i32(ctx.handle, C.c_void_p(pl.data_ptr()), C.c_void_p(bins.data_ptr()), n) == 0
    h = L.DenseHeader()
    sp = np.zeros(65536, dtype=np.float64)
    assert L.lib.skml_dense_info(ctx.handle, C.c_void_p(pl.data_ptr()), C.byref(h), sp.ctypes.data_as(L.dblp),
                                 65536) == 0
    xh = x.cpu().numpy()
    del x
    oq = O.quantize(xh, 256, int(p.seed))
    assert oq.bin_num == h.bin_num and oq.bin_num > 100
    assert (h.zero_idx, h.n) == (oq.zero_idx, n)
    assert np.float64(h.min).tobytes() == np.float64(oq.min).tobytes()
    assert np.float64(h.max).tobytes() == np.float64(oq.max).tobytes()
    assert np.array_equal(sp[: oq.bin_num - 1], oq.splits)
    gb = bins.cpu().numpy()
    assert np.array_equal(gb, oq.bins)
    assert np.array_equal(dec.cpu().numpy().view(np.uint64), oq.values()[oq.bins].view(np.uint64))


def test_f64_of_f32_values_equals_f32_path(gpu):
    """fp32 values widened to fp64 give the fp32 path's splits and bins (the reference converts
    every value to double anyway)."""
    n = 3 * 65536 + 999
    x32 = np.random.default_rng(5).standard_normal(n).astype(np.float32)
    a = gpu.QuantileQuantizer(256, seed=4)
    a.quantize(torch.from_numpy(x32).cuda())
    b = gpu.QuantileQuantizer(256, seed=4)
    b.quantize(torch.from_numpy(x32.astype(np.float64)).cuda())
    assert np.array_equal(a.getSplits(), b.getSplits())
    assert torch.equal(a.getBins(), b.getBins())


def test_f64_parallel_quantize_keeps_duplicates(gpu):
    x = _data64(50000, 9, "dups")
    gq = gpu.QuantileQuantizer(64, seed=5)
    gpu.Parallel.setParallelism(1)
    gq.parallelQuantize(torch.from_numpy(x).cuda())
    _check(gq, O.parallel_quantize(x, 64, threads=1, seed=5), x)


def test_f64_nan_raises(gpu):
    x = _data64(5000, 1)
    x[1234] = np.nan
    with pytest.raises(gpu.QuantileSketchException):
        gpu.QuantileQuantizer(16).quantize(torch.from_numpy(x).cuda())


def test_f64_write_object_matches_oracle(gpu):
    x = _data64(7000, 2)
    gq = gpu.QuantileQuantizer(256, seed=3)
    gq.quantize(torch.from_numpy(x).cuda())
    assert gq.writeObject() == O.quantize(x, 256, 3).write_ref()


# ------------------------------------------------------------------------------ uniform

def _uni_data(n, seed, kind):
    x = _data64(n, seed, "normal" if kind in ("nan", "zero_first", "neg_zero_first") else kind)
    rng = np.random.default_rng(seed + 1)
    if kind == "nan":
        x[rng.random(n) < 0.05] = np.nan
    elif kind == "zero_first":   # min is zero: the first zero decides its sign
        x = np.abs(x) + 1.0
        x[3] = 0.0
        x[7:] = np.where(rng.random(n - 7) < 0.1, -0.0, x[7:])
    elif kind == "neg_zero_first":
        x = np.abs(x) + 1.0
        x[3] = -0.0
        x[7:] = np.where(rng.random(n - 7) < 0.1, 0.0, x[7:])
    return x


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("kind", ["normal", "app", "nan", "zero_first", "neg_zero_first", "negative",
                                  "dups", "const", "special"])
def test_uniform_matches_oracle(gpu, wide, kind):
    n = 65536 * 3 + 321
    x = _uni_data(n, 17, kind)
    if not wide:
        x = x.astype(np.float32)
    gq = gpu.UniformQuantizer(256)
    gq.quantize(torch.from_numpy(x).cuda())
    oq = O.uniform_quantize(x.astype(np.float64), 256)
    _check(gq, oq, x)
    dec = gq.decode(dtype=torch.float64).cpu().numpy()
    assert np.array_equal(dec, oq.values()[oq.bins], equal_nan=True)


@pytest.mark.parametrize("bins", [2, 3, 4, 16, 255, 1000, 4096, 5000])
@pytest.mark.parametrize("wide", [False, True])
def test_uniform_bin_counts(gpu, bins, wide):
    x = _data64(100000, bins, "normal")
    if not wide:
        x = x.astype(np.float32)
    gq = gpu.UniformQuantizer(bins)
    gpu.Parallel.setParallelism(4)
    gq.parallelQuantize(torch.from_numpy(x).cuda())
    _check(gq, O.uniform_quantize(x.astype(np.float64), bins), x)


@pytest.mark.parametrize("vals", [[np.inf, 1.0, 2.0], [-np.inf, -1.0], [np.nan, np.nan],
                                  [-3.0, -1.0], [5.0, 0.0, -0.0, 2.0], [1e308, -1e308, 0.5], [7.0]])
@pytest.mark.parametrize("wide", [False, True])
def test_uniform_degenerate_ranges(gpu, vals, wide):
    """Java-literal indexOf on split tables that are NaN, infinite or overflowed."""
    x = np.array(vals * 300, dtype=np.float64 if wide else np.float32)
    if not wide and 1e308 in vals:
        pytest.skip("1e308 is not an fp32 value")
    gq = gpu.UniformQuantizer(8)
    gq.quantize(torch.from_numpy(x).cuda())
    _check(gq, O.uniform_quantize(x.astype(np.float64), 8), x)


def test_uniform_empty(gpu):
    gq = gpu.UniformQuantizer(8)
    gq.quantize(torch.empty(0, dtype=torch.float64, device="cuda"))
    oq = O.uniform_quantize(np.zeros(0), 8)
    assert gq.getBinNum() == oq.bin_num and gq.getZeroIdx() == oq.zero_idx
    assert np.array_equal(gq.getSplits(), oq.splits)


def test_uniform_write_object_and_compressor(gpu):
    x = _data64(9000, 4).astype(np.float32)
    comp = gpu.DenseVectorCompressor(gpu.QuantizationType.UNIFORM, 64)
    comp.compressDense(torch.from_numpy(x).cuda())
    oq = O.uniform_quantize(x.astype(np.float64), 64)
    assert comp.quantizer.quantizationType() == gpu.QuantizationType.UNIFORM
    assert comp.quantizer.writeObject() == oq.write_ref()
    dec = comp.decompressDense().cpu().numpy()
    assert np.array_equal(dec, oq.values()[oq.bins].astype(np.float32))

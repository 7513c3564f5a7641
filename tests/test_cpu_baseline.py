"""The CPU baseline bench.py times (oracle/cpu_baseline.cpp: the reference's dense encode on host
threads) computes what the oracle computes: QuantileQuantizer.quantize for 1 thread and
parallelQuantize + parallelQuantizeToBins (QuantileQuantizer.java:53-92, Quantizer.java:94-117) for
T threads, so the baseline is the reference algorithm, not a shortcut."""
import numpy as np
import pytest

from oracle import oracle as O


def _x(n, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n).astype(np.float32)
    if kind == "app":
        x[rng.random(n) >= 0.9] = 0.0
    elif kind == "zeros":
        r = rng.random(n)
        x[r < 0.2] = 0.0
        x[(r >= 0.2) & (r < 0.3)] = -0.0
    return x


@pytest.mark.parametrize("n,bins,kind", [(1, 256, "normal"), (255, 16, "normal"), (256, 256, "app"),
                                         (70001, 256, "zeros"), (2**18 + 333, 256, "app"), (100000, 4, "normal"),
                                         (50000, 1000, "normal")])
def test_one_thread_equals_quantize(n, bins, kind):
    x = _x(n, n, kind)
    h, sp, codes = O.cpu_encode(x, bins, seed=7, threads=1)
    oq = O.quantize(x.astype(np.float64), bins, 7)
    assert (h.bin_num, h.zero_idx, h.min, h.max) == (oq.bin_num, oq.zero_idx, oq.min, oq.max)
    assert np.array_equal(sp, oq.splits)
    assert np.array_equal(codes, ((oq.bins - 128) & 0xFF).astype(np.uint8))


@pytest.mark.parametrize("threads", [2, 3, 8])
@pytest.mark.parametrize("n", [1000, 2**17 + 12345])
def test_threads_equal_parallel_quantize(threads, n):
    x = _x(n, 3 * n + threads, "app")
    h, sp, codes = O.cpu_encode(x, 256, seed=11, threads=threads)
    oq = O.parallel_quantize(x.astype(np.float64), 256, threads=threads, seed=11)
    assert (h.bin_num, h.zero_idx, h.min, h.max) == (oq.bin_num, oq.zero_idx, oq.min, oq.max)
    assert np.array_equal(sp, oq.splits)
    assert np.array_equal(codes, ((oq.bins - 128) & 0xFF).astype(np.uint8))


def test_nan_rejected():
    x = _x(5000, 1)
    x[100] = np.nan
    for t in (1, 4):
        with pytest.raises(O.OracleError):
            O.cpu_encode(x, 256, 1, t)

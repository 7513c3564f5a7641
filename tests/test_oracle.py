"""CPU-only: pin the C restatement (oracle/) with hand-derived known-answer tests (SURVEY.md §8c
K1-K8, Appendix B JDK specs) and cross-check it against the independent numpy restatement.

The reference (Java) cannot run here and has no tests of its own, so these KATs -- worked by hand
from the Java sources and public JDK specifications -- are the only anchors ("parity unpinned"
against a live reference run).
"""
import struct

import numpy as np
import pytest

from oracle import np_oracle as N
from oracle import oracle as O


# ---------------------------------------------------------------- K6: java.util.Random spec
def test_java_random_kat():
    r = O.JavaRandom(42)
    assert [r.next_int() for _ in range(5)] == [-1170105035, 234785527, -1360544799, 205897768,
                                                1325939940]
    assert O.JavaRandom(0).next_int() == -1155484576
    assert O.JavaRandom(0).next_double() == 0.730967787376657
    assert O.JavaRandom(42).next_double() == 0.7275636800328681
    assert O.JavaRandom(0).next_gaussian() == pytest.approx(0.8025330637390305, abs=1e-15)


def test_java_random_next_int_bound_matches_numpy_restatement():
    for seed in (0, 1, 77, -5):
        a, b = O.JavaRandom(seed), N.JRandom(seed)
        for bound in (1, 2, 3, 7, 8, 10, 1000, 2**30 + 1):
            assert a.next_int(bound) == b.next_int(bound)


def test_lcg_jump_ahead_equals_stepping():
    for seed in (0, 9, 123456789):
        r = N.JRandom(seed)
        bits = [r.next_boolean() for _ in range(300)]
        assert bits == [bool(N.lcg_bit(seed, i)) for i in range(300)]
        assert bits[:50] == [bool(O.lib().orc_jr_bit_at(seed, i)) for i in range(50)]


# ---------------------------------------------------------------- K1: exact sketch for n <= 255
@pytest.mark.parametrize("n", [1, 2, 3, 17, 100, 255])
def test_small_n_sketch_is_exact(n):
    x = np.random.default_rng(n).standard_normal(n)
    parts = 256
    splits = O.sketch_quantiles(x, parts, seed=5)
    s = np.sort(x, kind="stable")
    frac = 1.0 / parts
    for i in range(parts - 1):
        rank = min(int(n * frac), n - 1)
        assert splits[i] == s[rank]
        frac += 1.0 / parts


# ---------------------------------------------------------------- K2: n = 2^m -> 129 bins
@pytest.mark.parametrize("m", [8, 10, 13])
def test_power_of_two_gives_129_bins(m):
    x = np.random.default_rng(m).standard_normal(2**m)
    q = O.quantize(x, 256, seed=11)
    assert q.bin_num == 129
    samples, weights, _, _ = O.sketch_summary(x, seed=11)
    assert len(samples) == 128
    assert np.array_equal(q.splits, samples)
    assert weights[-1] == 2**m


# ---------------------------------------------------------------- K3: indexOf == upper_bound
def _hdr_with(splits, mn, mx):
    q = O.quantize(np.array([0.0, 1.0]), 3, seed=0)  # any header, then overwrite its fields
    h = q.hdr
    h.bin_num = len(splits) + 1
    for i, s in enumerate(splits):
        h.splits[i] = s
    h.min, h.max = mn, mx
    # findZeroIdx (Quantizer.java:74-85)
    if mn > 0:
        h.zero_idx = 0
    elif mx < 0:
        h.zero_idx = h.bin_num - 1
    else:
        t = 0
        while t < h.bin_num - 1 and splits[t] < 0:
            t += 1
        h.zero_idx = t
    return O.OracleQuant(h, None)


@pytest.mark.parametrize("splits,mn,mx", [
    ([-1.0, 0.5, 0.7, 1.0], -2.0, 2.0),
    ([-3.0, -2.0, -2.0, -1.0, -1.0, -0.5], -4.0, 4.9e-324),   # negatives only, duplicates
    ([0.25, 0.5, 0.5, 0.5, 2.0, 8.0], 0.1, 9.0),               # positives only, duplicates
    ([-1.0, -0.0, 0.0, 1.0], -1.5, 1.5),                       # signed zeros
    ([0.0], -1.0, 1.0),
])
def test_index_of_is_upper_bound(splits, mn, mx):
    q = _hdr_with(splits, mn, mx)
    pts = sorted(set(splits + [mn, mx, 0.0, -0.0] + [s + d for s in splits for d in (-1e-9, 1e-9)]))
    pts = [p for p in pts if mn <= p <= mx]
    sp = np.array(splits)
    for p in pts:
        assert q.index_of(p) == int(np.searchsorted(sp, p, side="right")), p


# ---------------------------------------------------------------- K4: midpoints + MIN_VALUE max
def test_get_values_and_min_value_quirk():
    q = O.quantize(np.array([-3.0, -2.0, -1.0]), 4, seed=0)
    assert list(q.splits) == [-3.0, -2.0, -1.0]
    assert q.min == -3.0 and q.max == 4.9e-324          # Double.MIN_VALUE initial max
    assert q.zero_idx == 3                              # no split >= 0
    assert list(q.values()) == [-3.0, -2.5, -1.5, 0.5 * (-1.0 + 4.9e-324)]
    q = O.quantize(np.array([np.inf, np.inf]), 4, seed=0)
    assert q.min == 1.7976931348623157e308              # Double.MAX_VALUE initial min


# ---------------------------------------------------------------- K5: hashes (BKDR by hand)
def test_hash_kat_and_crosscheck():
    # BKDR(31): digits of 123 least-significant first: ((0*31+3)*31+2)*31+1 = 2946
    assert O.java_hash(3, 123, 1000) == 2946 % 1000
    assert O.java_hash(4, 123, 100000) == ((3 * 131 + 2) * 131 + 1)
    for hid in range(8):
        for key in (0, 1, 7, 99, 123456, 2**31 - 1, -5, 2**28 + 3):
            for size in (1, 3, 1000, 2**20 + 7):
                assert O.java_hash(hid, key, size) == N.java_hash(hid, key, size)


def test_pick_hashes_is_java_shuffle():
    for seed in (0, 3, 99):
        r = N.JRandom(seed)
        idx = list(range(8))
        for i in range(7, 0, -1):
            j = r.next_int(i + 1)
            idx[i], idx[j] = idx[j], idx[i]
        assert list(O.pick_hashes(seed, 2)) == idx[:2]


# ---------------------------------------------------------------- K7: DeltaAdaptive by hand
def test_delta_adaptive_kat_small():
    d = O.delta_encode([0, 1, 2, 3])
    # bits needed all 1 -> m=16 unary flags wins (t2 = 4); flags "10"x4, deltas 00 01 01 01
    assert d["num_intervals"] == 16 and d["flag_kind"] is True
    assert list(d["flag_words"]) == [0x55]
    assert list(d["delta_words"]) == [0xA8]
    assert d["n_flag_bits"] == 8 and d["n_delta_bits"] == 8


def test_delta_adaptive_kat_wide():
    d = O.delta_encode([5, 300, 70000])
    # deltas 5, 295, 69700 need 3, 9, 17 bits -> m=16 fixed 4-bit flags (t1 = 14.67)
    assert d["num_intervals"] == 16 and d["flag_kind"] is False
    assert list(d["flag_words"]) == [(1 << 3) | (1 << 5) | (1 << 8)]          # 0001 0100 1000
    pos = [1, 3, 5, 8, 11, 12, 13, 15, 19, 25, 29]  # 0101 | 0100100111 | 010001000001000100
    assert list(d["delta_words"]) == [sum(1 << p for p in pos)]
    assert d["n_delta_bits"] == 32
    assert list(d["decoded"]) == [5, 300, 70000]


def test_delta_adaptive_crosscheck_random():
    rng = np.random.default_rng(0)
    for n, span in ((1, 10), (50, 100), (3000, 2**20), (20000, 2**28)):
        keys = np.unique(rng.integers(0, span, n))
        a, b = O.delta_encode(keys), N.delta_encode(keys)
        for k in ("size", "num_intervals", "flag_kind", "n_flag_bits", "n_delta_bits"):
            assert a[k] == b[k]
        assert np.array_equal(a["flag_words"], b["flag_words"])
        assert np.array_equal(a["delta_words"], b["delta_words"])
        assert np.array_equal(a["decoded"], keys)


def test_delta_rejects_non_increasing_keys():
    with pytest.raises(O.OracleError):
        O.delta_encode([3, 3, 4])


# ---------------------------------------------------------------- K8: dense wire bytes
def test_quantizer_wire_bytes_kat():
    q = O.quantize(np.array([1.0, 2.0, 3.0]), 4, seed=0)
    assert list(q.bins) == [1, 2, 3] and q.zero_idx == 0
    be = lambda fmt, *v: struct.pack(">" + fmt, *v)
    want = (be("ii", 4, 3) + be("ddd", 1.0, 2.0, 3.0) + be("i", 0) + be("dd", 1.0, 3.0) +
            be("i", 3) + bytes([0x81, 0x82, 0x83]))
    assert q.write_ref() == want
    back = O.read_ref(want, 3)
    assert list(back.bins) == [1, 2, 3] and back.bin_num == 4


# ---------------------------------------------------------------- cross-check vs numpy tree
@pytest.mark.parametrize("n", [300, 511, 512, 1000, 4096, 9999, 2**15 + 77])
@pytest.mark.parametrize("seed", [0, 987654321])
def test_quantize_crosscheck_numpy_tree(n, seed):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n)
    x[rng.random(n) < 0.1] = 0.0
    x[rng.random(n) < 0.01] = -0.0
    q = O.quantize(x, 256, seed)
    r = N.quantize(x, 256, seed)
    assert q.bin_num == r["bin_num"] and q.zero_idx == r["zero_idx"]
    assert np.array_equal(q.splits, r["splits"])
    assert np.array_equal(q.bins, r["bins"])
    assert np.array_equal(q.values(), r["values"])


def test_parallel_quantize_single_thread_equals_sequential_before_dedup():
    x = np.random.default_rng(5).standard_normal(50000)
    a = O.parallel_quantize(x, 256, threads=1, seed=3)
    b = O.quantize(x, 256, seed=3)
    assert a.bin_num == 256                      # no Maths.unique in parallelQuantize
    uniq = a.splits[np.r_[True, a.splits[1:] != a.splits[:-1]]]
    assert np.array_equal(uniq, b.splits)
    # with duplicated splits indexOf still counts every split <= x (upper_bound)
    assert np.array_equal(a.bins, np.searchsorted(a.splits, x, side="right"))
    assert np.array_equal(b.bins, np.searchsorted(b.splits, x, side="right"))


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_parallel_quantize_split_ranks_within_epsilon(threads):
    x = np.random.default_rng(threads).standard_normal(200000)
    q = O.parallel_quantize(x, 64, threads=threads, seed=1)
    s = np.sort(x)
    for i, sp in enumerate(q.splits):
        rank = np.searchsorted(s, sp, side="left") / len(x)
        assert abs(rank - (i + 1) / 64) < 0.02
    assert np.array_equal(q.bins, np.searchsorted(q.splits, x, side="right"))


@pytest.mark.parametrize("n,threads,bins,seed", [
    (10000, 3, 64, 1), (1000, 4, 16, 2), (777, 8, 256, 4), (3, 5, 4, 5), (40000, 7, 256, 6),
    (256 * 9, 2, 32, 7), (256 * 9 + 5, 3, 32, 8), (70000, 2, 256, 9)])
def test_parallel_quantize_crosscheck_carry_buffer(n, threads, bins, seed):
    """C oracle vs the independent Python carry-buffer HeapQuantileSketch (update / merge)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n)
    if seed % 2:
        x[rng.random(n) < 0.2] = 0.0
        x[rng.random(n) < 0.05] = -0.0
    a = O.parallel_quantize(x, bins, threads=threads, seed=seed)
    b = N.parallel_quantize(x, bins, threads, seed)
    assert (a.bin_num, a.zero_idx, a.min, a.max) == (b["bin_num"], b["zero_idx"], b["min"], b["max"])
    assert np.array_equal(a.splits, b["splits"])
    assert np.array_equal(a.bins, b["bins"])


def test_nan_is_rejected():
    with pytest.raises(O.OracleError) as e:
        O.quantize(np.array([1.0, np.nan, 2.0]), 16)
    assert e.value.status == 2


def test_huffman_roundtrip_and_optimal_length():
    rng = np.random.default_rng(2)
    for vals in ([7], [1, 1, 1], rng.integers(0, 12, 5000), rng.geometric(0.3, 20000)):
        h = O.huffman_encode(vals)
        assert h["decode_status"] == 0
        assert np.array_equal(h["decoded"], np.asarray(vals, dtype=np.int32))
    # total length equals the optimal (Huffman) cost computed independently
    vals = rng.geometric(0.2, 10000)
    _, cnt = np.unique(vals, return_counts=True)
    import heapq
    heap = list(cnt.tolist())
    heapq.heapify(heap)
    cost = 0
    while len(heap) > 1:
        a, b = heapq.heappop(heap), heapq.heappop(heap)
        cost += a + b
        heapq.heappush(heap, a + b)
    assert O.huffman_encode(vals)["n_bits"] == cost


def test_sparse_roundtrip_properties():
    rng = np.random.default_rng(8)
    dim = 200000
    dense = np.where(rng.random(dim) < 0.1, rng.standard_normal(dim), 0.0)
    keys, vals = O.to_sparse(dense)
    s = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, seed=4, hash_seed=9)
    k2, b2 = s.restore()
    assert np.array_equal(k2, keys)                                   # P5
    z = s.q.zero_idx
    assert np.all(np.abs(b2 - z) <= np.abs(s.bins - z))              # P6
    assert s.group_size.sum() == len(keys)
    e = O.group_edges(z, s.q.bin_num, 8)
    assert np.array_equal(e, N.group_edges(z, s.q.bin_num, 8))


# ---------------------------------------------------------------- UniformQuantizer KATs
def _uniform_py(values, B):
    """UniformQuantizer.java:21-45 restated as plain Python loops (independent of the C oracle)."""
    mn, mx = 1.7976931348623157e308, 4.9e-324
    for v in values:
        if v < mn:
            mn = v
        if v > mx:
            mx = v
    step = (mx - mn) / B
    sp = [mn + step]
    for _ in range(1, B - 1):
        sp.append(sp[-1] + step)
    return mn, mx, sp


def test_uniform_kat():
    q = O.uniform_quantize(np.array([0.0, 1.0, 2.0, 3.0, 4.0]), 4)
    assert list(q.splits) == [1.0, 2.0, 3.0] and list(q.bins) == [0, 1, 2, 3, 3] and q.zero_idx == 0
    # all-negative input: max stays Double.MIN_VALUE (UniformQuantizer.java:25)
    q = O.uniform_quantize(np.array([-3.0, -1.0]), 2)
    assert q.max == 5e-324 and list(q.splits) == [-1.5] and list(q.bins) == [0, 1] and q.zero_idx == 1
    # the first zero decides the sign of a zero minimum; NaN is skipped, then binned by indexOf
    q = O.uniform_quantize(np.array([5.0, 0.0, -0.0, 2.0]), 4)
    assert np.signbit(q.min) == False and list(q.bins) == [3, 0, 0, 1]  # noqa: E712
    q = O.uniform_quantize(np.array([5.0, -0.0, 0.0, np.nan]), 4)
    assert np.signbit(q.min) and list(q.bins) == [3, 0, 0, 1]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_uniform_crosscheck_python_loops(seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(3000) * 10.0 ** int(rng.integers(-3, 4))
    x[rng.random(3000) < 0.01] = np.nan
    B = int(rng.integers(2, 300))
    q = O.uniform_quantize(x, B)
    mn, mx, sp = _uniform_py(x, B)
    assert q.min == mn and q.max == mx and list(q.splits) == sp
    assert all(q.bins[i] == q.index_of(x[i]) for i in range(0, 3000, 7))

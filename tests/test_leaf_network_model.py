"""CPU model of the sketch leaf's in-register sorting network (sketchml_amd/csrc/skml_device.hpp):
Batcher's odd-even merge sort over R registers with its first two merge levels replaced by the
3-input 4-sorter (v_min3 / v_med3 / v_max3_f32).  The order is Arrays.sort's total order
(-0.0 before +0.0; HeapQuantileSketch sorts its base buffer with it, HeapQuantileSketch.java:107-124),
which gfx950's v_min / v_max / v_min3 / v_med3 / v_max3_f32 follow (tools/ubench/min3_probe.hip,
run on the GPU: every operand order of 3-tuples and every 4-tuple over a signed-zero value set).

The model also states the VALU arithmetic of the change: a comparator is 2 ops (min + max), the
4-sorter 8 ops instead of 5 comparators, so R = 64 costs 1,054 ops instead of 1,086 per lane."""
import itertools

import numpy as np


def batcher_table(n):
    """OddEvenNet<N>::table() (skml_device.hpp), in the same loop order."""
    out = []
    p = 1
    while p < n:
        k = p
        while k >= 1:
            j = k % p
            while j < n - k:
                for i in range(min(k, n - j - k)):
                    if (i + j) // (2 * p) == (i + j + k) // (2 * p):
                        out.append((i + j, i + j + k))
                j += 2 * k
            k //= 2
        p *= 2
    return out


def key(x):
    """Total-order key of a float32: -0.0 < +0.0 (no NaN here: the leaf flags NaN before sorting)."""
    b = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return np.where(b >> 31, (~b) & 0xFFFFFFFF, b | 0x80000000)


def tmin(a, b):
    return np.where(key(a) <= key(b), a, b).astype(np.float32)


def tmax(a, b):
    return np.where(key(a) <= key(b), b, a).astype(np.float32)


def tmin3(a, b, c):
    return tmin(tmin(a, b), c)


def tmax3(a, b, c):
    return tmax(tmax(a, b), c)


def tmed3(a, b, c):
    return tmax(tmin(a, b), tmin(tmax(a, b), c))


def sort4_3in(a, b, c, d):
    p, q = tmin(a, b), tmax(a, b)
    return tmin3(p, c, d), tmin(tmed3(p, c, d), q), tmax(tmed3(q, c, d), p), tmax3(q, c, d)


def network_sort(v, use_sort4):
    """v: (R, lanes) float32 -> sorted along axis 0 by the leaf's network."""
    v = v.copy()
    R = v.shape[0]
    net = batcher_table(R)
    c0 = 0
    if use_sort4:
        for b in range(R // 4):
            v[4 * b], v[4 * b + 1], v[4 * b + 2], v[4 * b + 3] = sort4_3in(*v[4 * b: 4 * b + 4])
        c0 = 5 * (R // 4)
    for a, b in net[c0:]:
        v[a], v[b] = tmin(v[a], v[b]), tmax(v[a], v[b])
    return v


def test_batcher_counts_and_sort4_prefix():
    for R, want in ((8, 19), (16, 63), (32, 191), (64, 543)):
        net = batcher_table(R)
        assert len(net) == want
        c0 = 5 * (R // 4)
        assert all(a // 4 == b // 4 for a, b in net[:c0])  # the first two levels: inside blocks of 4
        assert net[c0][0] // 4 != net[c0][1] // 4
    assert 2 * 543 == 1086 and 2 * 543 - (10 - 8) * 16 == 1054


def test_sort4_3in_every_tuple_total_order():
    vals = np.array([-np.inf, -2.0, -1.0, -0.0, 0.0, 1.0, 2.0, np.inf], dtype=np.float32)
    tup = np.array(list(itertools.product(vals, repeat=4)), dtype=np.float32).T  # (4, 4096)
    got = np.stack(sort4_3in(*tup))
    want = np.take_along_axis(tup, np.argsort(key(tup), axis=0, kind="stable"), axis=0)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_network_with_sort4_base_sorts():
    rng = np.random.default_rng(7)
    for R in (8, 16, 64):
        x = rng.standard_normal((R, 512)).astype(np.float32)
        x[rng.random(x.shape) < 0.1] = 0.0
        x[rng.random(x.shape) < 0.1] = -0.0
        x[rng.random(x.shape) < 0.05] = 1.5  # duplicates
        want = np.take_along_axis(x, np.argsort(key(x), axis=0, kind="stable"), axis=0)
        for s4 in (False, True):
            got = network_sort(x, s4)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (R, s4)

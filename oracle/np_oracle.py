"""Independent pure-Python/numpy restatement of a subset of the reference algorithm.

TEST INFRASTRUCTURE ONLY.  Written separately from oracle/skml_oracle.c (different structure:
the sketch is expressed as the explicit binary merge tree over 256-element chunks that
SURVEY.md §8a-A2 derives, not as the carry-propagating buffer of HeapQuantileSketch.java), so
that agreement between the two is evidence for both.  Small inputs only (pure-Python loops).

Covered: java.util.Random, the sketch summary + getQuantiles(int), Maths.unique, findZeroIdx,
parallelQuantize (here as the carry-propagating buffer: the merge has no tree form),
bins = upper_bound(splits, x), getValues, the 8 hashes, calGroupEdges, DeltaAdaptive encode.
"""
from __future__ import annotations

import math
import struct

import numpy as np

MASK48 = (1 << 48) - 1
MULT = 0x5DEECE66D


# -------------------------------------------------------------------------- java.util.Random
class JRandom:
    def __init__(self, seed):
        self.s = (seed ^ MULT) & MASK48

    def next(self, bits):
        self.s = (self.s * MULT + 0xB) & MASK48
        v = self.s >> (48 - bits)
        v &= 0xFFFFFFFF
        return v - (1 << 32) if v >= (1 << 31) else v

    def next_boolean(self):
        return self.next(1) != 0

    def next_int(self, bound):
        r = self.next(31)
        m = bound - 1
        if bound & m == 0:
            return (bound * r) >> 31
        u = r
        while True:
            r = u % bound  # u >= 0 so Python % == Java %
            t = (u - r + m) & 0xFFFFFFFF
            if t < (1 << 31):
                return r
            u = self.next(31)


def lcg_bit(seed, idx):
    """next(1) of the idx-th call, by affine jump-ahead (s -> a*s + c) instead of stepping."""
    s = (seed ^ MULT) & MASK48
    a, c = MULT, 0xB
    steps = idx + 1
    while steps:
        if steps & 1:
            s = (a * s + c) & MASK48
        c = (a * c + c) & MASK48
        a = (a * a) & MASK48
        steps >>= 1
    return s >> 47


# -------------------------------------------------------------------------- sketch as a tree
def _total_key(x):
    u = struct.unpack("<Q", struct.pack("<d", x))[0]
    return (~u) & 0xFFFFFFFFFFFFFFFF if u >> 63 else u | (1 << 63)


def _merge_newer_first(older, newer):
    out = []
    i = j = 0
    while i < len(older) and j < len(newer):
        if older[i] < newer[j]:
            out.append(older[i]); i += 1
        else:
            out.append(newer[j]); j += 1
    return out + older[i:] + newer[j:]


def _popcount(x):
    return bin(x).count("1")


def _node(vals, seed, c0, level):
    """Node covering chunks [c0, c0 + 2**level): compaction bit of a node at `level` whose last
    chunk is c is stream index 2c - popcount(c) + level."""
    if level == 0:
        chunk = sorted(vals[c0 * 256:(c0 + 1) * 256], key=_total_key)
        c = c0
    else:
        half = 1 << (level - 1)
        left = _node(vals, seed, c0, level - 1)
        right = _node(vals, seed, c0 + half, level - 1)
        chunk = _merge_newer_first(left, right)
        c = c0 + (1 << level) - 1
    odd = lcg_bit(seed, 2 * c - _popcount(c) + level)
    return chunk[odd::2][:128]


def sketch_summary(values, seed):
    vals = [float(v) for v in values]
    n = len(vals)
    chunks = n // 256
    nodes = []  # (level, samples) with the most significant (oldest) tree first
    c0 = 0
    for lv in reversed(range(chunks.bit_length())):
        if chunks >> lv & 1:
            nodes.append((lv, _node(vals, seed, c0, lv)))
            c0 += 1 << lv
    samples, weights = [], []
    for lv, smp in sorted(nodes, key=lambda t: t[0]):  # copied lowest level first
        samples += smp
        weights += [2 << lv] * 128
    tail = sorted(vals[chunks * 256:], key=_total_key)
    samples += tail
    weights += [1] * len(tail)
    # blocky merge sort of 128-blocks == stable sort under IEEE `<` (left wins ties)
    order = sorted(range(len(samples)), key=lambda i: (samples[i] if samples[i] != 0 else 0.0, i))
    s = [samples[i] for i in order]
    w = [weights[i] for i in order]
    prefix = [0]
    for x in w:
        prefix.append(prefix[-1] + x)
    mn = min(vals, default=None)
    mx = max(vals, default=None)
    return s, prefix, mn, mx


def quantiles(samples, prefix, n, parts):
    out = []
    frac = 1.0 / parts
    step = 1.0 / parts
    for _ in range(parts - 1):
        rank = min(int(n * frac), n - 1)
        # largest idx with prefix[idx] <= rank
        lo, hi = 0, len(samples)
        while lo + 1 < hi:
            mid = (lo + hi) // 2
            if prefix[mid] <= rank:
                lo = mid
            else:
                hi = mid
        out.append(samples[lo])
        frac += step
    return out


def quantize(values, bin_num, seed):
    """QuantileQuantizer.quantize restated over the tree: returns dict(header..., bins)."""
    vals = np.asarray(values, dtype=np.float64)
    s, prefix, mn, mx = sketch_summary(vals, seed)
    n = len(vals)
    splits = quantiles(s, prefix, n, bin_num)
    uniq = [splits[0]] + [b for a, b in zip(splits, splits[1:]) if b != a]
    B = len(uniq) + 1
    vmin = min(mn, 1.7976931348623157e308)
    vmax = max(mx, 4.9e-324)
    if vmin > 0:
        zero = 0
    elif vmax < 0:
        zero = B - 1
    else:
        zero = next((t for t, sp in enumerate(uniq) if not sp < 0.0), B - 1)
    sp = np.array(uniq)
    bins = np.searchsorted(sp, vals, side="right").astype(np.int32)  # upper_bound
    lut = [0.5 * (vmin + uniq[0])] + [0.5 * (a + b) for a, b in zip(uniq, uniq[1:])] + \
          [0.5 * (uniq[-1] + vmax)]
    return dict(bin_num=B, zero_idx=zero, min=vmin, max=vmax, splits=sp, bins=bins,
                values=np.array(lut))


# -------------------------------------------------------------------------- parallelQuantize
class _CarrySketch:
    """HeapQuantileSketch as its carry-propagating buffer (update / merge /
    inPlacePropagation*, HeapQuantileSketch.java:74-124,186-228), levels as a dict."""

    def __init__(self, rng):
        self.rng = rng
        self.n = 0
        self.base = []
        self.levels = {}
        self.mn = 1.7976931348623157e308  # HeapQuantileSketch.java:67-68
        self.mx = 4.9e-324

    def _halve(self, buf):  # QSketchUtils.compactBuffer (QSketchUtils.java:45-51)
        odd = 1 if self.rng.next_boolean() else 0
        return buf[odd::2][:128]

    def _carry(self, node, level):  # levelwisePropagation (QSketchUtils.java:71-82)
        while level in self.levels:
            node = self._halve(_merge_newer_first(self.levels.pop(level), node))
            level += 1
        self.levels[level] = node

    def update(self, v):
        if v != v:
            raise ValueError("Encounter NaN value")
        self.mx = max(self.mx, v, key=_total_key)  # Math.max / Math.min: -0.0 < 0.0
        self.mn = min(self.mn, v, key=_total_key)
        self.base.append(v)
        self.n += 1
        if len(self.base) == 256:
            buf = sorted(self.base, key=_total_key)
            self.base = []
            self._carry(self._halve(buf), 0)

    def merge(self, o):
        if o.n == 0:
            return
        if self.n == 0:  # copy(other)
            self.n, self.base, self.levels = o.n, list(o.base), dict(o.levels)
            self.mn, self.mx = o.mn, o.mx
            return
        total = self.n + o.n
        for v in o.base:
            self.update(v)
        for lv in sorted(o.levels):  # inPlacePropagationMerge: the copied node is not halved
            self._carry(list(o.levels[lv]), lv)
        self.n = total
        self.mx = max(self.mx, o.mx, key=_total_key)
        self.mn = min(self.mn, o.mn, key=_total_key)


def parallel_quantize(values, bin_num, threads, seed):
    """QuantileQuantizer.parallelQuantize (QuantileQuantizer.java:53-92), the slice sketches
    run one after another and then merged in slice order, all from one Random(seed); no
    Maths.unique."""
    rng = JRandom(seed)
    vals = [float(v) for v in values]
    n = len(vals)
    per = n // threads
    sks = []
    for t in range(threads):
        lo = t * per
        hi = n if t == threads - 1 else lo + per
        sk = _CarrySketch(rng)
        for v in vals[lo:hi]:
            sk.update(v)
        sks.append(sk)
    acc = sks[0]
    for o in sks[1:]:
        acc.merge(o)
    samples, weights = [], []
    for lv in sorted(acc.levels):  # copyBuf2Arr: lowest level first, then the sorted base
        samples += acc.levels[lv]
        weights += [2 << lv] * 128
    tail = sorted(acc.base, key=_total_key)
    samples += tail
    weights += [1] * len(tail)
    order = sorted(range(len(samples)), key=lambda i: (samples[i] if samples[i] != 0 else 0.0, i))
    smp = [samples[i] for i in order]
    prefix = [0]
    for i in order:
        prefix.append(prefix[-1] + weights[i])
    splits = quantiles(smp, prefix, n, bin_num)
    vmin, vmax = acc.mn, acc.mx
    if vmin > 0:
        zero = 0
    elif vmax < 0:
        zero = bin_num - 1
    else:
        zero = next((t for t, sp in enumerate(splits) if not sp < 0.0), bin_num - 1)
    sp = np.array(splits)
    bins = np.searchsorted(sp, np.asarray(vals), side="right").astype(np.int32)
    return dict(bin_num=bin_num, zero_idx=zero, min=vmin, max=vmax, splits=sp, bins=bins)


# -------------------------------------------------------------------------- hashes
def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def _fold(c, size):
    r = int(math.fmod(c, size))  # truncating remainder like Java
    return r if r >= 0 else r + size


def hash_bj(c, size):
    c = _i32(c + 0x7ed55d16 + (c << 12))
    c = _i32((c ^ 0xc761c23c) ^ (c >> 19))
    c = _i32(c + 0x165667b1 + (c << 5))
    c = _i32((c + 0xd3a2646c) ^ (c << 9))
    c = _i32(c + 0xfd7046c5 + (c << 3))
    c = _i32((c ^ 0xb55a4f09) ^ (c >> 16))
    return _fold(c, size)


def hash_mix64(c, size):
    c = _i32(~c + (c << 21))
    c = _i32(c ^ (c >> 24))
    c = _i32(c + (c << 3) + (c << 8))
    c = _i32(c ^ (c >> 14))
    c = _i32(c + (c << 2) + (c << 4))
    c = _i32(c ^ (c >> 28))
    c = _i32(c + (c << 31))
    return _fold(c, size)


def hash_tw(c, size):
    c = _i32(~c + (c << 15))
    c = _i32(c ^ (c >> 12))
    c = _i32(c + (c << 2))
    c = _i32(c ^ (c >> 4))
    c = _i32(c * 2057)
    c = _i32(c ^ (c >> 16))
    return _fold(c, size)


def hash_bkdr(key, seed, size):
    c = 0
    while key != 0:
        c = _i32(seed * c + int(math.fmod(key, 10)))
        key = int(key / 10)
    return _fold(c, size)


def java_hash(hid, key, size):
    if hid == 0:
        return hash_bj(key, size)
    if hid == 1:
        return hash_mix64(key, size)
    if hid == 2:
        return hash_tw(key, size)
    return hash_bkdr(key, [31, 131, 267, 1313, 13131][hid - 3], size)


def group_edges(zero, B, g):
    if g == 2:
        return [zero, B]
    bpg = B // g
    if zero < bpg:
        e0 = zero
    elif zero % bpg < bpg // 2:
        e0 = bpg + zero % bpg
    else:
        e0 = zero % bpg
    e = [e0 + i * bpg for i in range(g - 1)] + [B]
    return e


# -------------------------------------------------------------------------- DeltaAdaptive
def delta_encode(keys):
    keys = [int(k) for k in keys]
    n = len(keys)
    deltas = [keys[0]] + [keys[i] - keys[i - 1] for i in range(1, n)]
    need = [1 if (i == 0 and d == 0) else d.bit_length() for i, d in enumerate(deltas)]
    prob = [0.0] * 32
    for b in need:
        prob[b] += 1.0
    prob = [p / n for p in prob]
    best, bm, bk = 32.0, 1, False
    for m in (2, 4, 8, 16):
        b = 32 // m
        ip = [0.0] * m
        s = 0.0
        for i in range(m):
            for j in range(b):
                ip[i] += prob[i * b + j]
            s += (i + 1) * ip[i]
        t1 = s * b + (m.bit_length() - 1)
        if t1 < best:
            best, bm, bk = t1, m, False
        t2 = s * (b + 1) + 1
        if t2 < best:
            best, bm, bk = t2, m, True
    bpi = 32 // bm
    flags, dbits = [], []
    for d, nb in zip(deltas, need):
        iv = -(-nb // bpi)
        if not bk:
            nf = bm.bit_length() - 1
            flags += [(iv - 1) >> (nf - 1 - i) & 1 for i in range(nf)]
        else:
            flags += [1] * iv + [0]
        w = bpi * iv
        dbits += [d >> (w - 1 - i) & 1 for i in range(w)]

    def words(bits):
        nw = (len(bits) + 63) // 64
        out = [0] * nw
        for p, b in enumerate(bits):
            if b:
                out[p >> 6] |= 1 << (p & 63)
        while out and out[-1] == 0:
            out.pop()
        return np.array(out, dtype=np.uint64)

    return dict(size=n, num_intervals=bm, flag_kind=bk, n_flag_bits=len(flags),
                n_delta_bits=len(dbits), flag_words=words(flags), delta_words=words(dbits))

"""ctypes binding of the C restatement in oracle/skml_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker.  The product package (sketchml_amd) never imports it.
See skml_oracle.h for the pinning status ("parity unpinned" against a live reference run).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libskml_oracle.so")

i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
dblp = C.POINTER(C.c_double)
u8p = C.POINTER(C.c_uint8)
u64p = C.POINTER(C.c_uint64)


class QuantHeader(C.Structure):
    _fields_ = [("bin_num", C.c_int32), ("n", C.c_int32), ("zero_idx", C.c_int32),
                ("min", C.c_double), ("max", C.c_double), ("splits", C.c_double * 65536)]


class JRandom(C.Structure):
    _fields_ = [("s", C.c_uint64), ("have_gauss", C.c_int), ("gauss", C.c_double)]


class Delta(C.Structure):
    _fields_ = [("size", C.c_int32), ("num_intervals", C.c_int32), ("flag_kind", C.c_int32),
                ("n_flag_bits", C.c_int64), ("n_delta_bits", C.c_int64),
                ("n_flag_longs", C.c_int32), ("n_delta_longs", C.c_int32),
                ("flag_words", u64p), ("delta_words", u64p)]


class Huffman(C.Structure):
    _fields_ = [("n_items", C.c_int32), ("item_value", i32p), ("item_bits", i32p),
                ("item_nbits", i32p), ("n_bits", C.c_int64), ("n_longs", C.c_int32),
                ("words", u64p), ("size", C.c_int32)]


class Sparse(C.Structure):
    _fields_ = [("q", QuantHeader), ("group_num", C.c_int32), ("row_num", C.c_int32),
                ("col_ratio", C.c_double), ("edges", C.c_int32 * 64),
                ("group_size", C.c_int32 * 64), ("col_num", C.c_int32 * 64),
                ("hash_ids", (C.c_int32 * 8) * 64), ("tables", i32p * 64),
                ("deltas", Delta * 64)]


def _build():
    if not os.path.exists(_SO):
        subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        _build()
        L = C.CDLL(_SO)
        L.orc_jr_seed.argtypes = [C.POINTER(JRandom), C.c_int64]
        L.orc_jr_next.argtypes = [C.POINTER(JRandom), C.c_int]
        L.orc_jr_next.restype = C.c_int32
        L.orc_jr_next_int.argtypes = [C.POINTER(JRandom)]
        L.orc_jr_next_int.restype = C.c_int32
        L.orc_jr_next_int_bound.argtypes = [C.POINTER(JRandom), C.c_int32]
        L.orc_jr_next_int_bound.restype = C.c_int32
        L.orc_jr_next_boolean.argtypes = [C.POINTER(JRandom)]
        L.orc_jr_next_double.argtypes = [C.POINTER(JRandom)]
        L.orc_jr_next_double.restype = C.c_double
        L.orc_jr_next_gaussian.argtypes = [C.POINTER(JRandom)]
        L.orc_jr_next_gaussian.restype = C.c_double
        L.orc_jr_bit_at.argtypes = [C.c_int64, C.c_int64]
        L.orc_quantize.argtypes = [dblp, C.c_int32, C.c_int32, C.c_int64, C.POINTER(QuantHeader), i32p]
        L.orc_parallel_quantize.argtypes = [dblp, C.c_int32, C.c_int32, C.c_int32, C.c_int64,
                                            C.POINTER(QuantHeader), i32p]
        L.orc_uniform_quantize.argtypes = [dblp, C.c_int32, C.c_int32, C.POINTER(QuantHeader), i32p]
        L.orc_quantize_header_f32.argtypes = [C.POINTER(C.c_float), C.c_int64, C.c_int32, C.c_int64,
                                              C.POINTER(QuantHeader)]
        L.orc_index_of_many_f32.argtypes = [C.POINTER(QuantHeader), C.POINTER(C.c_float), C.c_int64, i32p]
        L.orc_index_of_many_f32.restype = None
        L.orc_index_of.argtypes = [C.POINTER(QuantHeader), C.c_double]
        L.orc_index_of.restype = C.c_int32
        L.orc_get_values.argtypes = [C.POINTER(QuantHeader), dblp]
        L.orc_times_by.argtypes = [C.POINTER(QuantHeader), C.c_double]
        L.orc_write_ref.argtypes = [C.POINTER(QuantHeader), i32p, u8p, C.c_int64]
        L.orc_write_ref.restype = C.c_int64
        L.orc_read_ref.argtypes = [u8p, C.c_int64, C.POINTER(QuantHeader), i32p, C.c_int32]
        L.orc_sketch_summary.argtypes = [dblp, C.c_int64, C.c_int64, dblp, i64p, C.c_int64, dblp, dblp]
        L.orc_sketch_summary.restype = C.c_int64
        L.orc_sketch_quantiles.argtypes = [dblp, C.c_int64, C.c_int64, C.c_int32, dblp]
        L.orc_count_nnz.argtypes = [dblp, C.c_int64]
        L.orc_count_nnz.restype = C.c_int64
        L.orc_to_sparse.argtypes = [dblp, C.c_int64, i32p, dblp]
        L.orc_to_sparse.restype = C.c_int64
        L.orc_hash.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        L.orc_hash.restype = C.c_int32
        L.orc_pick_hashes.argtypes = [C.c_int64, C.c_int32, i32p]
        L.orc_group_edges.argtypes = [C.c_int32, C.c_int32, C.c_int32, i32p]
        L.orc_group_edges.restype = C.c_int
        L.orc_delta_encode.argtypes = [i32p, C.c_int32, C.POINTER(Delta)]
        L.orc_delta_decode.argtypes = [C.POINTER(Delta), i32p]
        L.orc_delta_free.argtypes = [C.POINTER(Delta)]
        L.orc_huffman_encode.argtypes = [i32p, C.c_int32, C.POINTER(Huffman)]
        L.orc_huffman_decode.argtypes = [C.POINTER(Huffman), i32p]
        L.orc_huffman_free.argtypes = [C.POINTER(Huffman)]
        L.orc_sparse_compress.argtypes = [i32p, dblp, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                          C.c_double, C.c_int64, C.c_int64, C.POINTER(Sparse), i32p]
        L.orc_sparse_compress_q.argtypes = [i32p, dblp, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                            C.c_double, C.c_int64, C.c_int64, C.c_int32, C.POINTER(Sparse), i32p]
        L.orc_sparse_restore.argtypes = [C.POINTER(Sparse), i32p, i32p]
        L.orc_sparse_restore.restype = C.c_int32
        L.orc_sparse_free.argtypes = [C.POINTER(Sparse)]
        L.orc_bench_dense_encode.argtypes = [C.POINTER(C.c_float), C.c_int32, C.c_int32, C.c_int64,
                                             C.c_int, u8p]
        L.orc_bench_dense_encode.restype = C.c_double
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


class OracleError(RuntimeError):
    def __init__(self, status, what):
        super().__init__(f"oracle {what} failed with status {status}")
        self.status = status


# ---------------------------------------------------------------- java.util.Random
class JavaRandom:
    def __init__(self, seed: int):
        self._r = JRandom()
        lib().orc_jr_seed(C.byref(self._r), seed)

    def next_int(self, bound=None):
        if bound is None:
            return lib().orc_jr_next_int(C.byref(self._r))
        return lib().orc_jr_next_int_bound(C.byref(self._r), bound)

    def next_bits(self, bits):
        return lib().orc_jr_next(C.byref(self._r), bits)

    def next_boolean(self):
        return bool(lib().orc_jr_next_boolean(C.byref(self._r)))

    def next_double(self):
        return lib().orc_jr_next_double(C.byref(self._r))

    def next_gaussian(self):
        return lib().orc_jr_next_gaussian(C.byref(self._r))


# ---------------------------------------------------------------- dense quantizer
class OracleQuant:
    """Result of QuantileQuantizer.quantize: header fields + int32 bins."""

    def __init__(self, hdr: QuantHeader, bins):
        self.hdr = hdr
        self.bin_num = hdr.bin_num
        self.n = hdr.n
        self.zero_idx = hdr.zero_idx
        self.min = hdr.min
        self.max = hdr.max
        self.splits = np.array(hdr.splits[: max(hdr.bin_num - 1, 0)], dtype=np.float64)
        self.bins = bins

    def values(self):
        out = np.zeros(self.bin_num, dtype=np.float64)
        lib().orc_get_values(C.byref(self.hdr), _p(out, dblp))
        return out

    def index_of(self, x: float) -> int:
        return lib().orc_index_of(C.byref(self.hdr), float(x))

    def write_ref(self) -> bytes:
        need = lib().orc_write_ref(C.byref(self.hdr), _p(self.bins, i32p), None, 0)
        buf = np.zeros(need, dtype=np.uint8)
        lib().orc_write_ref(C.byref(self.hdr), _p(self.bins, i32p), _p(buf, u8p), need)
        return buf.tobytes()


def quantize(values, bin_num=256, seed=0) -> OracleQuant:
    v = np.ascontiguousarray(values, dtype=np.float64)
    hdr = QuantHeader()
    bins = np.zeros(max(len(v), 1), dtype=np.int32)
    st = lib().orc_quantize(_p(v, dblp), len(v), bin_num, seed, C.byref(hdr), _p(bins, i32p))
    if st:
        raise OracleError(st, "quantize")
    return OracleQuant(hdr, bins[: len(v)])


def quantize_header_f32(values, bin_num=256, seed=0) -> OracleQuant:
    """QuantileQuantizer.quantize's header (sketch, getQuantiles, Maths.unique, findZeroIdx) of float
    values widened to double, without the bins: the full-size tests take those slice by slice from
    index_of_many_f32 (bins is None here)."""
    v = np.ascontiguousarray(values, dtype=np.float32)
    hdr = QuantHeader()
    st = lib().orc_quantize_header_f32(v.ctypes.data_as(C.POINTER(C.c_float)), len(v), bin_num, seed, C.byref(hdr))
    if st:
        raise OracleError(st, "quantize_header_f32")
    return OracleQuant(hdr, None)


def index_of_many_f32(oq: OracleQuant, values) -> np.ndarray:
    """Quantizer.quantizeToBins of a float slice against oq's header (ctypes releases the GIL, so
    slices can run on a thread pool)."""
    v = np.ascontiguousarray(values, dtype=np.float32)
    out = np.empty(len(v), dtype=np.int32)
    lib().orc_index_of_many_f32(C.byref(oq.hdr), v.ctypes.data_as(C.POINTER(C.c_float)), len(v), _p(out, i32p))
    return out


def uniform_quantize(values, bin_num=256) -> OracleQuant:
    """UniformQuantizer.quantize (quantization/UniformQuantizer.java:21-45)."""
    v = np.ascontiguousarray(values, dtype=np.float64)
    hdr = QuantHeader()
    bins = np.zeros(max(len(v), 1), dtype=np.int32)
    st = lib().orc_uniform_quantize(_p(v, dblp), len(v), bin_num, C.byref(hdr), _p(bins, i32p))
    if st:
        raise OracleError(st, "uniform_quantize")
    return OracleQuant(hdr, bins[: len(v)])


def parallel_quantize(values, bin_num=256, threads=4, seed=0) -> OracleQuant:
    v = np.ascontiguousarray(values, dtype=np.float64)
    hdr = QuantHeader()
    bins = np.zeros(max(len(v), 1), dtype=np.int32)
    st = lib().orc_parallel_quantize(_p(v, dblp), len(v), bin_num, threads, seed, C.byref(hdr),
                                     _p(bins, i32p))
    if st:
        raise OracleError(st, "parallel_quantize")
    return OracleQuant(hdr, bins[: len(v)])


def read_ref(buf: bytes, n_cap: int) -> OracleQuant:
    a = np.frombuffer(buf, dtype=np.uint8).copy()
    hdr = QuantHeader()
    bins = np.zeros(max(n_cap, 1), dtype=np.int32)
    st = lib().orc_read_ref(_p(a, u8p), len(a), C.byref(hdr), _p(bins, i32p), n_cap)
    if st:
        raise OracleError(st, "read_ref")
    return OracleQuant(hdr, bins[: hdr.n])


def sketch_summary(values, seed=0):
    v = np.ascontiguousarray(values, dtype=np.float64)
    cap = 64 * 128 + 256 + 1
    s = np.zeros(cap, dtype=np.float64)
    w = np.zeros(cap, dtype=np.int64)
    mn, mx = C.c_double(), C.c_double()
    ns = lib().orc_sketch_summary(_p(v, dblp), len(v), seed, _p(s, dblp), _p(w, i64p), cap,
                                  C.byref(mn), C.byref(mx))
    if ns < 0:
        raise OracleError(-ns, "sketch_summary")
    return s[:ns], w[: ns + 1], mn.value, mx.value


def sketch_quantiles(values, parts, seed=0):
    v = np.ascontiguousarray(values, dtype=np.float64)
    out = np.zeros(max(parts - 1, 1), dtype=np.float64)
    st = lib().orc_sketch_quantiles(_p(v, dblp), len(v), seed, parts, _p(out, dblp))
    if st:
        raise OracleError(st, "sketch_quantiles")
    return out[: parts - 1]


# ---------------------------------------------------------------- sparse pieces
def to_sparse(dense):
    d = np.ascontiguousarray(dense, dtype=np.float64)
    nnz = lib().orc_count_nnz(_p(d, dblp), len(d))
    k = np.zeros(max(nnz, 1), dtype=np.int32)
    v = np.zeros(max(nnz, 1), dtype=np.float64)
    lib().orc_to_sparse(_p(d, dblp), len(d), _p(k, i32p), _p(v, dblp))
    return k[:nnz], v[:nnz]


def java_hash(hash_id, key, size):
    return lib().orc_hash(hash_id, key, size)


def pick_hashes(seed, rows):
    ids = np.zeros(8, dtype=np.int32)
    lib().orc_pick_hashes(seed, rows, _p(ids, i32p))
    return ids[:rows]


def group_edges(zero_idx, bin_num, group_num):
    e = np.zeros(group_num, dtype=np.int32)
    lib().orc_group_edges(zero_idx, bin_num, group_num, _p(e, i32p))
    return e


def _words(ptr, n):
    return np.array([ptr[i] for i in range(n)], dtype=np.uint64) if n else np.zeros(0, np.uint64)


def delta_encode(keys):
    k = np.ascontiguousarray(keys, dtype=np.int32)
    d = Delta()
    st = lib().orc_delta_encode(_p(k, i32p), len(k), C.byref(d))
    if st:
        raise OracleError(st, "delta_encode")
    res = dict(size=d.size, num_intervals=d.num_intervals, flag_kind=bool(d.flag_kind),
               n_flag_bits=d.n_flag_bits, n_delta_bits=d.n_delta_bits,
               flag_words=_words(d.flag_words, d.n_flag_longs),
               delta_words=_words(d.delta_words, d.n_delta_longs))
    out = np.zeros(len(k), dtype=np.int32)
    lib().orc_delta_decode(C.byref(d), _p(out, i32p))
    res["decoded"] = out
    lib().orc_delta_free(C.byref(d))
    return res


def huffman_encode(values):
    v = np.ascontiguousarray(values, dtype=np.int32)
    h = Huffman()
    st = lib().orc_huffman_encode(_p(v, i32p), len(v), C.byref(h))
    if st:
        raise OracleError(st, "huffman_encode")
    res = dict(items=[(h.item_value[i], h.item_bits[i], h.item_nbits[i]) for i in range(h.n_items)],
               n_bits=h.n_bits, words=_words(h.words, h.n_longs), size=h.size)
    out = np.zeros(max(len(v), 1), dtype=np.int32)
    st = lib().orc_huffman_decode(C.byref(h), _p(out, i32p))
    res["decoded"] = out[: len(v)]
    res["decode_status"] = st
    lib().orc_huffman_free(C.byref(h))
    return res


class OracleSparse:
    def __init__(self, s: Sparse, bins):
        self._s = s
        self.bins = bins
        self.q = OracleQuant(s.q, bins)
        self.group_num = s.group_num
        self.edges = np.array(s.edges[: s.group_num], dtype=np.int32)
        self.group_size = np.array(s.group_size[: s.group_num], dtype=np.int32)
        self.col_num = np.array(s.col_num[: s.group_num], dtype=np.int32)
        self.hash_ids = np.array([list(s.hash_ids[g][: s.row_num]) for g in range(s.group_num)],
                                 dtype=np.int32)
        self.tables = []
        self.deltas = []
        for g in range(s.group_num):
            if not s.tables[g]:
                self.tables.append(None)
                self.deltas.append(None)
                continue
            nt = s.row_num * s.col_num[g]
            self.tables.append(np.ctypeslib.as_array(s.tables[g], shape=(nt,)).copy())
            d = s.deltas[g]
            self.deltas.append(dict(size=d.size, num_intervals=d.num_intervals,
                                    flag_kind=bool(d.flag_kind), n_flag_bits=d.n_flag_bits,
                                    n_delta_bits=d.n_delta_bits,
                                    flag_words=np.ctypeslib.as_array(d.flag_words, shape=(max(d.n_flag_longs, 1),))[: d.n_flag_longs].copy(),
                                    delta_words=np.ctypeslib.as_array(d.delta_words, shape=(max(d.n_delta_longs, 1),))[: d.n_delta_longs].copy()))

    def restore(self):
        nnz = int(self.group_size.sum())
        k = np.zeros(max(nnz, 1), dtype=np.int32)
        b = np.zeros(max(nnz, 1), dtype=np.int32)
        m = lib().orc_sparse_restore(C.byref(self._s), _p(k, i32p), _p(b, i32p))
        return k[:m], b[:m]

    def __del__(self):
        try:
            lib().orc_sparse_free(C.byref(self._s))
        except Exception:
            pass


def sparse_compress(keys, vals, bin_num=256, group_num=8, row_num=2, col_ratio=0.3, seed=0,
                    hash_seed=0, uniform=False) -> OracleSparse:
    k = np.ascontiguousarray(keys, dtype=np.int32)
    v = np.ascontiguousarray(vals, dtype=np.float64)
    s = Sparse()
    bins = np.zeros(max(len(k), 1), dtype=np.int32)
    st = lib().orc_sparse_compress_q(_p(k, i32p), _p(v, dblp), len(k), bin_num, group_num, row_num,
                                     col_ratio, seed, hash_seed, 1 if uniform else 0, C.byref(s), _p(bins, i32p))
    if st:
        lib().orc_sparse_free(C.byref(s))
        raise OracleError(st, "sparse_compress")
    return OracleSparse(s, bins[: len(k)])


EPS = 1e-8  # Maths.EPS (ml/.../util/Maths.scala)


def _java_int_two_thirds(dim):
    """dim * 2 / 3 in Java int arithmetic (SparseDoubleGradient.scala:47)."""
    v = (dim * 2) & 0xFFFFFFFF
    v = v - (1 << 32) if v >= 1 << 31 else v
    return int(v / 3)


class GradientSumError(ValueError):
    """The IllegalArgumentException of SparseDoubleGradient's constructor (a `require`)."""


def gradient_sum(restored, dim, scale=1.0):
    """Gradient.sum (ml/.../gradient/Gradient.scala:44-49) over SketchGradients of sparse form, each
    given as its restored (keys, values) in Sort.merge order (values = quantValues[bins] after
    timesBy).  Returns (sum, forms), forms[p] = "dense" | "sparse".

    sum = new DenseDoubleGradient(dim) (+0.0 everywhere); for each payload in order
    sum.plusBy(p.toAuto) (DenseDoubleGradient.scala:38): SketchGradient.toSparse
    (SketchGradient.scala:62-68) builds SparseDoubleGradient(dim, keys, values), whose constructor
    requires strictly increasing keys in [0, dim) (SparseDoubleGradient.scala:9-14; a repeated
    key raises); toAuto (:45-48) takes toDense when countNNZ (|v| > EPS, :28-34) exceeds
    dim * 2 / 3 in Java int arithmetic.  toDense (:36-42) writes the live values into zeros and
    plusBy(dense) (DenseDoubleGradient.scala:10-14) adds every entry (so -0.0 sums become +0.0);
    plusBy(sparse) (:16-22) adds each value at its key.  Then timesBy(scale) when scale != 1 (the
    exchange's 1/P)."""
    out = np.zeros(dim, dtype=np.float64)
    forms = []
    lim = _java_int_two_thirds(dim)
    for k, v in restored:
        k = np.asarray(k, dtype=np.int64)
        v = np.asarray(v, dtype=np.float64)
        if len(k) == 0:
            raise GradientSumError("head of empty list (SparseDoubleGradient.scala:11)")
        if k[0] < 0:
            raise GradientSumError(f"requirement failed: Negative index: {k[0]}.")
        if len(k) > 1 and not np.all(k[1:] > k[:-1]):
            raise GradientSumError("requirement failed: Indices are not strictly increasing")
        if k[-1] >= dim:
            raise GradientSumError(f"requirement failed: Index {k[-1]} out of bounds for gradient of dimension {dim}")
        live = np.abs(v) > EPS
        if int(live.sum()) > lim:
            out += 0.0
            out[k[live]] += v[live]
            forms.append("dense")
        else:
            out[k] += v
            forms.append("sparse")
    if scale != 1.0:
        out *= scale
    return out, forms


def bench_dense_encode(x_f32, bin_num=256, seed=0, reps=1):
    x = np.ascontiguousarray(x_f32, dtype=np.float32)
    codes = np.zeros(len(x), dtype=np.uint8)
    t = lib().orc_bench_dense_encode(x.ctypes.data_as(C.POINTER(C.c_float)), len(x), bin_num, seed,
                                     reps, _p(codes, u8p))
    return t, codes


# ---------------------------------------------------------------- CPU baseline (bench.py)
class CpbHeader(C.Structure):
    _fields_ = [("bin_num", C.c_int32), ("zero_idx", C.c_int32), ("status", C.c_int32), ("pad", C.c_int32),
                ("min", C.c_double), ("max", C.c_double)]


_cpb = None


def cpb_lib():
    """oracle/cpu_baseline.cpp: the reference's dense encode (quantize / parallelQuantize +
    (parallel)quantizeToBins) in optimised C++ on host threads -- bench.py's CPU baseline."""
    global _cpb
    if _cpb is None:
        so = os.path.join(_HERE, "_build", "libskml_cpubase.so")
        if not os.path.exists(so):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = C.CDLL(so)
        fp = C.POINTER(C.c_float)
        L.cpb_encode.argtypes = [fp, C.c_int32, C.c_int32, C.c_int64, C.c_int32, u8p, C.POINTER(CpbHeader), dblp]
        L.cpb_encode.restype = C.c_int
        L.cpb_bench.argtypes = [fp, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_int32, u8p]
        L.cpb_bench.restype = C.c_double
        _cpb = L
    return _cpb


def cpu_encode(x_f32, bin_num=256, seed=0, threads=1):
    """One CPU-baseline encode: (header, splits, 1-byte (bin - 128) codes)."""
    x = np.ascontiguousarray(x_f32, dtype=np.float32)
    codes = np.zeros(max(len(x), 1), dtype=np.uint8)
    h = CpbHeader()
    sp = np.zeros(max(bin_num - 1, 1), dtype=np.float64)
    st = cpb_lib().cpb_encode(x.ctypes.data_as(C.POINTER(C.c_float)), len(x), bin_num, seed, threads,
                              _p(codes, u8p), C.byref(h), _p(sp, dblp))
    if st:
        raise OracleError(st, "cpu_encode")
    return h, sp[: h.bin_num - 1], codes[: len(x)]


def cpu_bench(x_f32, bin_num=256, seed=0, threads=1, reps=1):
    """Wall seconds of `reps` CPU-baseline encodes."""
    x = np.ascontiguousarray(x_f32, dtype=np.float32)
    codes = np.zeros(max(len(x), 1), dtype=np.uint8)
    return cpb_lib().cpb_bench(x.ctypes.data_as(C.POINTER(C.c_float)), len(x), bin_num, seed, threads, reps,
                               _p(codes, u8p))

"""Sparse codec over the HIP kernels: SparseVectorCompressor, GroupedMinMaxSketch and
DeltaAdaptiveEncoder, mirroring sample/SparseVectorCompressor.java:22-148,
sketch/frequency/GroupedMinMaxSketch.java:19-172 and binary/DeltaAdaptiveEncoder.java:17-188.

The encoded state is a library-owned skml_sparse object in device memory (quantizer payload,
MinMaxSketch tables, DeltaAdaptive bit streams); the views below copy group data to the host
only when asked (parity checks, serialisation).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .constants import Parallel
from .context import get_context
from .exceptions import SketchMLException, check
from .quantization import Quantizer, QuantizationType


def _params(bin_num, group_num, row_num, col_ratio, seed, hash_seed, dedup=True, uniform=False, parallelism=1):
    p = _lib.Params()
    _lib.lib.skml_params_default(C.byref(p))
    p.bin_num = int(bin_num)
    p.group_num = int(group_num)
    p.row_num = int(row_num)
    p.col_ratio = float(col_ratio)
    p.seed = int(seed)
    p.hash_seed = int(hash_seed)
    p.dedup = 1 if dedup else 0
    p.quant_type = 1 if uniform else 0  # SKML_UNIFORM / SKML_QUANTILE
    p.parallelism = int(parallelism)
    return p


class SparsePayload:
    """Owner of one skml_sparse handle (GroupedMinMaxSketch + the values' quantizer)."""

    def __init__(self, handle: C.c_void_p, device: int, rows: int):
        self.handle = handle
        self.device = device
        self.rows = rows

    def _ctx(self):
        return get_context(self.device)

    def nnz(self) -> int:
        v = C.c_int64()
        check(_lib.lib.skml_sparse_nnz(self.handle, C.byref(v)), "sparse_nnz")
        return v.value

    def quant_header(self):
        hdr = _lib.DenseHeader()
        splits = np.zeros(_lib.SKML_MAX_BINS, dtype=np.float64)
        check(_lib.lib.skml_sparse_quant_info(self.handle, C.byref(hdr), splits.ctypes.data_as(_lib.dblp),
                                              len(splits)), "sparse_quant_info")
        return hdr, splits[: max(hdr.bin_num - 1, 0)].copy()

    def values(self) -> np.ndarray:
        hdr, _ = self.quant_header()
        out = np.zeros(max(hdr.bin_num, 1), dtype=np.float64)
        check(_lib.lib.skml_sparse_values(self.handle, out.ctypes.data_as(_lib.dblp), len(out)), "sparse_values")
        return out[: hdr.bin_num]

    def group(self, g: int) -> dict:
        info = _lib.SparseGroup()
        check(_lib.lib.skml_sparse_group_info(self._ctx().handle, self.handle, g, C.byref(info), None, None, None),
              "group_info")
        res = dict(size=info.size)
        if info.size == 0:
            return res
        table = np.zeros(max(info.col_num * self.rows, 1), dtype=np.int32)
        fw = np.zeros((info.n_flag_bits + 63) // 64 + 1, dtype=np.uint64)
        dw = np.zeros((info.n_delta_bits + 63) // 64 + 1, dtype=np.uint64)
        check(_lib.lib.skml_sparse_group_info(
            self._ctx().handle, self.handle, g, C.byref(info), table.ctypes.data_as(_lib.i32p),
            fw.ctypes.data_as(C.POINTER(C.c_uint64)), dw.ctypes.data_as(C.POINTER(C.c_uint64))), "group_info")

        def trim(w):  # BitSet.toLongArray: up to the last non-zero word
            nz = np.nonzero(w)[0]
            return w[: nz[-1] + 1] if len(nz) else w[:0]

        res.update(col_num=info.col_num, hash_ids=list(info.hash_ids)[: self.rows], num_intervals=info.num_intervals,
                   flag_kind=bool(info.flag_kind), n_flag_bits=info.n_flag_bits, n_delta_bits=info.n_delta_bits,
                   table=table, flag_words=trim(fw), delta_words=trim(dw))
        return res

    def restore(self, dtype=torch.float32):
        """GroupedMinMaxSketch.restore + SparseVectorCompressor.decompressSparse: device keys
        (int32) and values quantValues[bin] (fp32 of the doubles, or the doubles themselves with
        dtype=torch.float64, as the reference returns them).  A restored bin outside quantValues
        raises SketchMLException, as the reference's array lookup throws."""
        n = self.nnz()
        dev = torch.device("cuda", self.device)
        wide = dtype == torch.float64
        keys = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        vals = torch.empty(max(n, 1), dtype=torch.float64 if wide else torch.float32, device=dev)
        fn = _lib.lib.skml_sparse_decode_f64 if wide else _lib.lib.skml_sparse_decode_f32
        check(fn(self._ctx().handle, self.handle, C.c_void_p(keys.data_ptr()), C.c_void_p(vals.data_ptr())),
              "sparse_decode")
        return keys[:n], vals[:n]

    def serialize(self) -> bytes:
        """GroupedMinMaxSketch.writeObject field stream (layout in DESIGN.md / skml_sparse_serialize)."""
        need = C.c_size_t()
        check(_lib.lib.skml_sparse_serialize(self._ctx().handle, self.handle, None, 0, C.byref(need)), "serialize")
        buf = np.empty(max(need.value, 1), dtype=np.uint8)
        check(_lib.lib.skml_sparse_serialize(self._ctx().handle, self.handle, buf.ctypes.data_as(_lib.u8p),
                                             need.value, C.byref(need)), "serialize")
        return buf[: need.value].tobytes()

    def restore_bins(self):
        """GroupedMinMaxSketch.restore (GroupedMinMaxSketch.java:123-146): device keys and int32
        bins in Sort.merge order."""
        n = self.nnz()
        dev = torch.device("cuda", self.device)
        keys = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        bins = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        check(_lib.lib.skml_sparse_restore_bins(self._ctx().handle, self.handle, C.c_void_p(keys.data_ptr()),
                                                C.c_void_p(bins.data_ptr())), "sparse_restore")
        return keys[:n], bins[:n]

    @classmethod
    def deserialize(cls, data: bytes, quant_values=None, device=None) -> "SparsePayload":
        """GroupedMinMaxSketch.readObject of the stream serialize() writes; quant_values (the
        SparseVectorCompressor.quantValues doubles) make restore() return values as well."""
        dev = torch.cuda.current_device() if device is None else torch.device(device).index
        try:
            arr = np.frombuffer(data, dtype=np.uint8)  # zero copy for buffer objects (read only: a const stream)
        except TypeError:
            arr = np.frombuffer(bytes(data), dtype=np.uint8)  # any iterable of ints, as bytes() accepts
        qv = None if quant_values is None else np.ascontiguousarray(quant_values, dtype=np.float64)
        h = C.c_void_p()
        check(_lib.lib.skml_sparse_deserialize(
            get_context(dev).handle, arr.ctypes.data_as(_lib.u8p), len(arr),
            qv.ctypes.data_as(_lib.dblp) if qv is not None else None, 0 if qv is None else len(qv), C.byref(h)),
            "readObject")
        rows = int.from_bytes(arr[4:8].tobytes(), "big", signed=True) if len(arr) >= 8 else 0
        return cls(h, dev, rows)

    def times_by(self, x: float) -> None:
        check(_lib.lib.skml_sparse_times_by(self.handle, float(x)), "sparse_times_by")

    def export_bytes(self) -> int:
        n = C.c_size_t()
        check(_lib.lib.skml_sparse_export_bytes(self.handle, C.byref(n)), "sparse_export_bytes")
        return n.value

    def export(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """The payload as one relocatable device blob (skml_sparse_export; the unit the RCCL
        all-gather moves).  `out`: a 256-byte aligned uint8 device tensor of >= export_bytes()."""
        nb = self.export_bytes()
        if out is None:
            out = torch.empty(nb, dtype=torch.uint8, device=torch.device("cuda", self.device))
        if out.numel() * out.element_size() < nb:
            raise SketchMLException(f"export buffer of {out.numel()} bytes < {nb}")
        check(_lib.lib.skml_sparse_export(self._ctx().handle, self.handle, C.c_void_p(out.data_ptr()), nb),
              "sparse_export")
        return out

    @classmethod
    def from_blob(cls, blob: torch.Tensor, nbytes: int | None = None) -> "SparsePayload":
        """skml_sparse_import: an owned payload from a blob in device memory (checked first)."""
        dev = blob.device.index
        h = C.c_void_p()
        n = blob.numel() * blob.element_size() if nbytes is None else int(nbytes)
        check(_lib.lib.skml_sparse_import(get_context(dev).handle, C.c_void_p(blob.data_ptr()), n, C.byref(h)),
              "sparse_import")
        pl = cls(h, dev, 0)
        pl.rows = int(np.frombuffer(blob[256 + 4: 256 + 8].cpu().numpy().tobytes(), dtype=np.int32)[0])
        return pl

    def __del__(self):
        try:
            if self.handle:
                _lib.lib.skml_sparse_free(self.handle)
                self.handle = None
        except Exception:
            pass


def decode_sum(blobs: torch.Tensor, nblobs: int, stride: int, dim: int, scale: float = 1.0,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Gradient.sum (ml/gradient/Gradient.scala:44-49) of `nblobs` exported sparse payloads laid out
    `stride` bytes apart: a float64 dense sum of length dim, payloads added in order (then scaled
    when scale != 1).  skml_sparse_decode_sum_f64.  Like SketchGradient.toSparse's
    SparseDoubleGradient constructor, a payload whose restored keys repeat (a key in two groups)
    or leave [0, dim), or that restores no keys at all (the constructor reads indices.head),
    raises SketchMLException."""
    dev = blobs.device
    if out is None:
        out = torch.empty(max(int(dim), 1), dtype=torch.float64, device=dev)
    check(_lib.lib.skml_sparse_decode_sum_f64(get_context(dev.index).handle, C.c_void_p(blobs.data_ptr()),
                                              int(nblobs), int(stride), int(dim), float(scale),
                                              C.c_void_p(out.data_ptr())), "sparse_decode_sum")
    return out[: int(dim)]


def _as_device(t, dtype, device=None):
    t = torch.as_tensor(t)
    if device is None:
        device = t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
    return t.to(device=device, dtype=dtype).contiguous()


def _values_dtype(values):
    """fp64 values (the reference's double[]) stay fp64; everything else is binned as fp32."""
    dt = values.dtype if isinstance(values, torch.Tensor) else np.asarray(values).dtype
    return torch.float64 if dt in (torch.float64, np.float64) else torch.float32


def encode_sparse(keys, values, bin_num=Quantizer.DEFAULT_BIN_NUM, group_num=8, row_num=2, col_ratio=0.3,
                  seed=0, hash_seed=0, dedup=True, uniform=False, parallelism=1) -> SparsePayload:
    """SparseVectorCompressor.compressSparse (SparseVectorCompressor.java:52-67).  Double values
    go through skml_sparse_encode_kv_f64 (the quantizer sketches the doubles themselves, as the
    Java double[] path does); float values through the fp32 kernels."""
    v = _as_device(values, _values_dtype(values))
    k = _as_device(keys, torch.int32, v.device)
    if k.numel() != v.numel():
        raise SketchMLException(
            f"Lengths of key array and value array do not match: {k.numel()}, {v.numel()}")
    dev = v.device.index
    ctx = get_context(dev)
    p = _params(bin_num, group_num, row_num, col_ratio, seed, hash_seed, dedup, uniform, parallelism)
    h = C.c_void_p()
    fn = _lib.lib.skml_sparse_encode_kv_f64 if v.dtype == torch.float64 else _lib.lib.skml_sparse_encode_kv_f32
    check(fn(ctx.handle, C.c_void_p(k.data_ptr()), C.c_void_p(v.data_ptr()), k.numel(), C.byref(p), C.byref(h)),
          "sparse_encode")
    return SparsePayload(h, dev, int(row_num))


def encode_dense_as_sparse(dense, bin_num=Quantizer.DEFAULT_BIN_NUM, group_num=8, row_num=2, col_ratio=0.3,
                           seed=0, hash_seed=0, uniform=False) -> SparsePayload:
    """SketchGradient.fromSparse after DenseDoubleGradient.toSparse (|x| > 1e-8), on device; a
    float64 gradient (DenseDoubleGradient.values itself) is compacted and binned as doubles."""
    x = _as_device(dense, _values_dtype(dense))
    dev = x.device.index
    ctx = get_context(dev)
    p = _params(bin_num, group_num, row_num, col_ratio, seed, hash_seed, True, uniform)
    h = C.c_void_p()
    fn = _lib.lib.skml_sparse_encode_f64 if x.dtype == torch.float64 else _lib.lib.skml_sparse_encode_f32
    check(fn(ctx.handle, C.c_void_p(x.data_ptr()), x.numel(), C.byref(p), C.byref(h)), "sparse_encode")
    return SparsePayload(h, dev, int(row_num))


def to_sparse(dense):
    """DenseDoubleGradient.countNNZ + toSparse (ml/gradient/DenseDoubleGradient.scala:64-89);
    float64 input keeps float64 values."""
    x = _as_device(dense, _values_dtype(dense))
    ctx = get_context(x.device.index)
    keys = torch.empty(max(x.numel(), 1), dtype=torch.int32, device=x.device)
    vals = torch.empty(max(x.numel(), 1), dtype=x.dtype, device=x.device)
    nnz = C.c_int64()
    fn = _lib.lib.skml_sparse_compact_f64 if x.dtype == torch.float64 else _lib.lib.skml_sparse_compact_f32
    check(fn(ctx.handle, C.c_void_p(x.data_ptr()), x.numel(),
                                           C.c_void_p(keys.data_ptr()), C.c_void_p(vals.data_ptr()),
                                           C.byref(nnz)), "sparse_compact")
    return keys[: nnz.value], vals[: nnz.value]


class GroupedMinMaxSketch:
    """frequency/GroupedMinMaxSketch.java:19-172.  create(keys, values) runs the quantizer and
    the grouped sketch in one device call (the reference passes the quantizer's bins)."""

    DEFAULT_MINMAXSKETCH_GROUP_NUM = 8
    DEFAULT_MINMAXSKETCH_COL_RATIO = 0.3

    def __init__(self, groupNum=DEFAULT_MINMAXSKETCH_GROUP_NUM, rowNum=2, colRatio=DEFAULT_MINMAXSKETCH_COL_RATIO,
                 binNum=Quantizer.DEFAULT_BIN_NUM, seed=0, hashSeed=0):
        self.groupNum = int(groupNum)
        self.rowNum = int(rowNum)
        self.colRatio = float(colRatio)
        self.binNum = int(binNum)
        self.seed = seed
        self.hashSeed = hashSeed
        self.zeroValue = None
        self.payload: SparsePayload | None = None

    def create(self, keys, values, dedup=True, uniform=False, parallelism=1) -> None:
        self.payload = encode_sparse(keys, values, self.binNum, self.groupNum, self.rowNum, self.colRatio,
                                     self.seed, self.hashSeed, dedup, uniform, parallelism)
        hdr, _ = self.payload.quant_header()
        self.binNum = hdr.bin_num
        self.zeroValue = hdr.zero_idx

    def restore(self):
        """GroupedMinMaxSketch.restore (GroupedMinMaxSketch.java:123-146): (keys, int32 bins)."""
        return self.payload.restore_bins()

    def getGroup(self, g: int) -> dict:
        return self.payload.group(g)

    def writeObject(self) -> bytes:
        return self.payload.serialize()

    @classmethod
    def readObject(cls, data: bytes, device=None) -> "GroupedMinMaxSketch":
        """GroupedMinMaxSketch.readObject (GroupedMinMaxSketch.java:161-172); restore() then gives
        (keys, bins) like the reference's restore()."""
        pl = SparsePayload.deserialize(data, None, device)
        head = np.frombuffer(bytes(data[:28]), dtype=">i4", count=2)
        sk = cls(int(head[0]), int(head[1]))
        sk.colRatio = float(np.frombuffer(bytes(data[8:16]), dtype=">f8")[0])
        sk.binNum, sk.zeroValue = (int(v) for v in np.frombuffer(bytes(data[16:24]), dtype=">i4"))
        sk.payload = pl
        return sk


class DeltaAdaptiveEncoder:
    """binary/DeltaAdaptiveEncoder.java:17-188 (BinaryEncoder, base/BinaryEncoder.java:6-11)."""

    def __init__(self):
        self.size = 0
        self.numIntervals = 0
        self.flagKind = False
        self.nFlagBits = 0
        self.nDeltaBits = 0
        self.flagWords = None   # device uint64 (BitSet.toLongArray)
        self.deltaWords = None

    def encode(self, values) -> None:
        k = _as_device(values, torch.int32)
        n = k.numel()
        ctx = get_context(k.device.index)
        cap = n + 2  # >= the longer of the two streams in 64-bit words (<= 49 bits per key)
        fw = torch.zeros(cap, dtype=torch.int64, device=k.device)
        dw = torch.zeros(cap, dtype=torch.int64, device=k.device)
        m, kind = C.c_int32(), C.c_int32()
        nf, nd = C.c_int64(), C.c_int64()
        check(_lib.lib.skml_delta_encode(ctx.handle, C.c_void_p(k.data_ptr()), n, C.byref(m), C.byref(kind),
                                         C.byref(nf), C.byref(nd), C.c_void_p(fw.data_ptr()),
                                         C.c_void_p(dw.data_ptr()), cap), "delta_encode")
        self.size = n
        self.numIntervals = m.value
        self.flagKind = bool(kind.value)
        self.nFlagBits = nf.value
        self.nDeltaBits = nd.value

        def trim(w, bits):
            w = w[: (bits + 63) // 64]
            nz = torch.nonzero(w).flatten()
            return w[: int(nz[-1].item()) + 1] if nz.numel() else w[:0]

        self.flagWords = trim(fw, nf.value)
        self.deltaWords = trim(dw, nd.value)

    def decode(self) -> torch.Tensor:
        dev = self.flagWords.device if self.flagWords is not None else torch.device("cuda")
        out = torch.empty(max(self.size, 1), dtype=torch.int32, device=dev)
        ctx = get_context(dev.index)
        fw = self.flagWords if self.flagWords.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
        dw = self.deltaWords if self.deltaWords.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
        check(_lib.lib.skml_delta_decode(ctx.handle, self.size, self.numIntervals, int(self.flagKind),
                                         C.c_void_p(fw.data_ptr()), self.flagWords.numel(),
                                         C.c_void_p(dw.data_ptr()), self.deltaWords.numel(),
                                         C.c_void_p(out.data_ptr())), "delta_decode")
        return out[: self.size]


class SparseVectorCompressor:
    """sample/SparseVectorCompressor.java:22-148."""

    def __init__(self, quantType=QuantizationType.QUANTILE, quantBinNum: int = Quantizer.DEFAULT_BIN_NUM,
                 mmSketchGroupNum: int = GroupedMinMaxSketch.DEFAULT_MINMAXSKETCH_GROUP_NUM,
                 mmSketchRowNum: int = 2,
                 mmSketchColRatio: float = GroupedMinMaxSketch.DEFAULT_MINMAXSKETCH_COL_RATIO,
                 seed: int = 0, hashSeed: int = 0):
        if str(quantType) not in ("QUANTILE", "UNIFORM"):
            raise SketchMLException(f"Unrecognizable quantization type: {quantType}")
        self.quantType = quantType
        self.quantBinNum = int(quantBinNum)
        self.mmSketchGroupNum = int(mmSketchGroupNum)
        self.mmSketchRowNum = int(mmSketchRowNum)
        self.mmSketchColRatio = float(mmSketchColRatio)
        self.seed = seed
        self.hashSeed = hashSeed
        self._size = 0
        self.mmSketches: GroupedMinMaxSketch | None = None

    def _compress(self, keys, values, dedup, parallelism=1):
        self.mmSketches = GroupedMinMaxSketch(self.mmSketchGroupNum, self.mmSketchRowNum, self.mmSketchColRatio,
                                              self.quantBinNum, self.seed, self.hashSeed)
        self.mmSketches.create(keys, values, dedup, str(self.quantType) == "UNIFORM", parallelism)
        self._size = self.mmSketches.payload.nnz()

    def compressDense(self, values) -> None:
        v = _as_device(values, torch.float32)
        keys = torch.arange(v.numel(), dtype=torch.int32, device=v.device)
        self._compress(keys, v, True)

    def compressSparse(self, keys, values) -> None:
        self._compress(keys, values, True)

    def parallelCompressDense(self, values) -> None:
        v = _as_device(values, torch.float32)
        keys = torch.arange(v.numel(), dtype=torch.int32, device=v.device)
        self._compress(keys, v, False, Parallel.getParallelism())

    def parallelCompressSparse(self, keys, values) -> None:
        """parallelQuantize with T = Constants.Parallel.getParallelism() slice sketches (no
        Maths.unique) + parallelCreate (same groups), SparseVectorCompressor.java:80-98."""
        self._compress(keys, values, False, Parallel.getParallelism())

    def decompressSparse(self):
        """SparseVectorCompressor.decompressSparse (SparseVectorCompressor.java:118-126): keys and
        quantValues[bins] (fp32 on the device)."""
        return self.mmSketches.payload.restore()

    def decompressDense(self) -> torch.Tensor:
        """Dense array of length maxKey + 1 (SparseVectorCompressor.java:106-114)."""
        keys, vals = self.decompressSparse()
        n = int(keys.max().item()) + 1 if keys.numel() else 1
        out = torch.zeros(n, dtype=torch.float32, device=vals.device)
        out[keys.long()] = vals
        return out

    def timesBy(self, x: float) -> None:
        if self.mmSketches is not None and self.mmSketches.payload is not None:
            self.mmSketches.payload.times_by(x)

    def size(self) -> float:
        return float(self._size)

    def memoryBytes(self) -> int:
        """28 + 8 * binNum + the serialised GroupedMinMaxSketch (SparseVectorCompressor.java:142-147;
        the field stream without Java object-stream framing)."""
        res = 28
        if self.mmSketches is not None and self.mmSketches.payload is not None:
            res += 8 * len(self.mmSketches.payload.values())
            res += len(self.mmSketches.writeObject())
        return res

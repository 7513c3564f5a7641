"""Quantizer / QuantileQuantizer over the HIP codec.

Mirrors base/Quantizer.java:18-228 and quantization/QuantileQuantizer.java:18-99: the same
method names, argument meaning and exceptions, with the gradient held on the GPU.  The encoded
state is one device payload (header + split table + packed codes, include/skml.h); getBins()
materialises int32 bins on demand.
"""
from __future__ import annotations

import ctypes as C
import struct
from enum import Enum

import numpy as np
import torch

from . import _lib
from .constants import Parallel
from .context import alloc_aligned, as_device_values, get_context
from .exceptions import QuantileSketchException, SketchMLException, check


class QuantizationType(Enum):
    UNIFORM = "UNIFORM"
    QUANTILE = "QUANTILE"

    def __str__(self):
        return self.value


class Quantizer:
    """base/Quantizer.java:18-228."""

    DEFAULT_BIN_NUM = 256

    def __init__(self, binNum: int = DEFAULT_BIN_NUM, seed: int = 0, deferred: bool = False):
        """deferred=True: quantize() only queues the encode on the stream and returns (no host
        synchronisation); the header is read, and a NaN input raises QuantileSketchException, at
        the first getter (getBins, getSplits, writeObject, ...) or at the next quantize(),
        whichever comes first.  The next quantize() of a QuantileQuantizer reads the previous
        header first (one host synchronisation per call) because QuantileQuantizer.java:42 carries
        the binNum that Maths.unique reduced into the next encode; back-to-back deferred quantile
        encodes therefore synchronise once per call, and only the first encode of a series runs
        with no synchronisation at all.  The UniformQuantizer never lowers binNum (no Maths.unique,
        UniformQuantizer.java:21-45), so its deferred encodes skip that read and never
        synchronise.  Every encode gets a payload buffer of its own, so a `payload` reference
        taken earlier keeps its bytes.  The default keeps the reference's eager behaviour."""
        self.binNum = int(binNum)
        self.seed = int(seed)
        self._deferred = bool(deferred)
        self.n = 0
        self.payload = None          # torch.uint8 device tensor
        self.device = None
        self._hdr = None
        self._splits = None
        self._bins = None
        self._wide = False           # input was fp64 (decode() then returns float64)

    # ---- abstract surface ----
    def quantize(self, values) -> None:
        raise NotImplementedError

    def parallelQuantize(self, values) -> None:
        raise NotImplementedError

    def quantizationType(self) -> QuantizationType:
        raise NotImplementedError

    @staticmethod
    def newQuantizer(qtype, binNum: int, seed: int = 0) -> "Quantizer":
        """Quantizer.newQuantizer (Quantizer.java:126-136)."""
        if str(qtype) == "QUANTILE":
            return QuantileQuantizer(binNum, seed)
        if str(qtype) == "UNIFORM":
            return UniformQuantizer(binNum, seed)
        raise SketchMLException(f"Unrecognizable quantization type: {qtype}")

    # ---- device payload plumbing ----
    def _ctx(self):
        return get_context(self.device)

    def _load_header(self):
        if self._hdr is None:
            hdr = _lib.DenseHeader()
            splits = np.zeros(_lib.SKML_MAX_BINS, dtype=np.float64)
            st = _lib.lib.skml_dense_info(self._ctx().handle, C.c_void_p(self.payload.data_ptr()),
                                          C.byref(hdr), splits.ctypes.data_as(_lib.dblp), len(splits))
            check(st, "quantize")
            self._hdr = hdr
            self._splits = splits[: hdr.bin_num - 1].copy()
            self.binNum = hdr.bin_num
            self._x = None  # a deferred encode has consumed its input
        return self._hdr

    _ENTRY = {(False, False): "skml_dense_encode_f32", (False, True): "skml_dense_encode_f64",
              (True, False): "skml_dense_encode_uniform_f32", (True, True): "skml_dense_encode_uniform_f64"}

    def _encode(self, values, dedup: bool, uniform: bool = False, threads: int = 1):
        if self._deferred and self.payload is not None and self._hdr is None and not uniform:
            try:
                self._load_header()  # the previous encode's effective binNum (and its NaN status)
            except QuantileSketchException:
                self.payload = None  # reported once; the next quantize starts clean
                raise
        x = as_device_values(values, self.device)
        self._wide = x.dtype == torch.float64
        self.device = x.device
        self.n = x.numel()
        if self.binNum <= 1:
            raise QuantileSketchException(f"Invalid partition number: {self.binNum}")
        nbytes = _lib.lib.skml_dense_payload_bytes(self.n, self.binNum)
        if nbytes == 0:
            raise SketchMLException(f"bad quantizer arguments n={self.n} binNum={self.binNum}")
        self.payload = alloc_aligned(nbytes, x.device)
        p = _lib.Params()
        _lib.lib.skml_params_default(C.byref(p))
        p.bin_num = self.binNum
        p.seed = self.seed
        p.dedup = 1 if dedup else 0
        if threads > 1 and not uniform:
            fn = _lib.lib.skml_dense_encode_parallel_f64 if self._wide else _lib.lib.skml_dense_encode_parallel_f32
            st = fn(self._ctx().handle, C.c_void_p(x.data_ptr()), self.n, threads, C.byref(p),
                    C.c_void_p(self.payload.data_ptr()), nbytes)
        else:
            fn = getattr(_lib.lib, self._ENTRY[(uniform, self._wide)])
            st = fn(self._ctx().handle, C.c_void_p(x.data_ptr()), self.n, C.byref(p),
                    C.c_void_p(self.payload.data_ptr()), nbytes)
        check(st, "quantize")
        self._hdr = None
        self._bins = None
        self._x = x  # keep the input alive until the stream has consumed it
        if not self._deferred:
            self._load_header()  # surfaces NaN as QuantileSketchException, like update() throws

    def _encode_sharded(self, values, shard_sizes, shard: int, records: torch.Tensor, dedup: bool = False):
        """Quantise shard `shard` of one logical gradient against the split table of the merged
        shard sketches (skml_dense_encode_sharded_f32); records = all shards' records in order."""
        x = as_device_values(values, self.device)
        self._wide = x.dtype == torch.float64
        self.device = x.device
        self.n = x.numel()
        sizes = np.ascontiguousarray(shard_sizes, dtype=np.int64)
        nbytes = _lib.lib.skml_dense_payload_bytes(self.n, self.binNum)
        if nbytes == 0:
            raise SketchMLException(f"bad quantizer arguments n={self.n} binNum={self.binNum}")
        self.payload = alloc_aligned(nbytes, x.device)
        p = _lib.Params()
        _lib.lib.skml_params_default(C.byref(p))
        p.bin_num = self.binNum
        p.seed = self.seed
        p.dedup = 1 if dedup else 0
        fn = _lib.lib.skml_dense_encode_sharded_f64 if self._wide else _lib.lib.skml_dense_encode_sharded_f32
        st = fn(self._ctx().handle, C.c_void_p(x.data_ptr()), self.n, sizes.ctypes.data_as(_lib.i64p), len(sizes),
                int(shard), C.c_void_p(records.data_ptr()), C.byref(p), C.c_void_p(self.payload.data_ptr()), nbytes)
        check(st, "quantize")
        self._hdr = None
        self._bins = None
        self._x = (x, records)
        self._load_header()
        self._x = None

    # ---- Quantizer getters ----
    def getValues(self) -> np.ndarray:
        """Quantizer.getValues (Quantizer.java:39-47): bin midpoints in double."""
        h = self._load_header()
        s = self._splits
        ns = h.bin_num - 1
        res = np.empty(h.bin_num, dtype=np.float64)
        res[0] = 0.5 * (h.min + s[0])
        for i in range(1, ns):
            res[i] = 0.5 * (s[i - 1] + s[i])
        res[ns] = 0.5 * (s[ns - 1] + h.max)
        return res

    def indexOf(self, x: float) -> int:
        """Quantizer.indexOf (Quantizer.java:49-72) on the host (one value)."""
        h = self._load_header()
        s = self._splits
        B = h.bin_num
        if x < s[0]:
            return 0
        if x >= s[B - 2]:
            return B - 1
        lo = hi = h.zero_idx
        if x < 0.0:
            lo = 0
        else:
            hi = B - 2
        while lo + 1 < hi:
            mid = (lo + hi) >> 1
            if s[mid] > x:
                if mid == 0 or s[mid - 1] <= x:
                    return mid
                hi = mid
            else:
                lo = mid
        mid = (lo + hi) >> 1
        return mid + 1 if s[mid] <= x else mid

    def getBins(self) -> torch.Tensor:
        """Quantizer.getBins: int32 bins materialised on the device."""
        if self._bins is None:
            self._load_header()
            b = torch.empty(self.n, dtype=torch.int32, device=self.device)
            check(_lib.lib.skml_dense_bins_i32(self._ctx().handle, C.c_void_p(self.payload.data_ptr()),
                                               C.c_void_p(b.data_ptr()), self.n), "getBins")
            self._bins = b
        return self._bins

    def getBinNum(self) -> int:
        return self._load_header().bin_num if self.payload is not None else self.binNum

    def getN(self) -> int:
        return self.n

    def getSplits(self) -> np.ndarray:
        self._load_header()
        return self._splits.copy()

    def getZeroIdx(self) -> int:
        return self._load_header().zero_idx

    def getMin(self) -> float:
        return self._load_header().min

    def getMax(self) -> float:
        return self._load_header().max

    def codeBits(self) -> int:
        return self._load_header().code_bits

    def timesBy(self, x: float) -> None:
        """Quantizer.timesBy (Quantizer.java:119-124)."""
        self._load_header()
        check(_lib.lib.skml_dense_times_by(self._ctx().handle, C.c_void_p(self.payload.data_ptr()),
                                           float(x)), "timesBy")
        self._hdr = None

    def decode(self, out: torch.Tensor = None, dtype=None) -> torch.Tensor:
        """values[bins[i]] on the device (DenseVectorCompressor.decompressDense): fp32 for fp32
        input, fp64 (the reference's double[]) for fp64 input or dtype=torch.float64."""
        self._load_header()
        if dtype is None:
            dtype = out.dtype if out is not None else (torch.float64 if self._wide else torch.float32)
        if out is None:
            out = torch.empty(self.n, dtype=dtype, device=self.device)
        if out.dtype != dtype or out.numel() != self.n or not out.is_contiguous():
            raise SketchMLException("decode: output must be a contiguous tensor of n values of the decode dtype")
        fn = _lib.lib.skml_dense_decode_f64 if dtype == torch.float64 else _lib.lib.skml_dense_decode_f32
        check(fn(self._ctx().handle, C.c_void_p(self.payload.data_ptr()), C.c_void_p(out.data_ptr()), self.n),
              "decode")
        return out

    # ---- java serialisation field stream ----
    def writeObject(self) -> bytes:
        """Quantizer.writeObject (Quantizer.java:184-203) field stream, big-endian."""
        self._load_header()
        n = C.c_size_t()
        ctx = self._ctx().handle
        pl = C.c_void_p(self.payload.data_ptr())
        check(_lib.lib.skml_dense_serialize_ref(ctx, pl, None, 0, C.byref(n)), "writeObject")
        buf = np.zeros(n.value, dtype=np.uint8)
        check(_lib.lib.skml_dense_serialize_ref(ctx, pl, buf.ctypes.data_as(_lib.u8p), n.value,
                                                C.byref(n)), "writeObject")
        return buf.tobytes()

    @classmethod
    def readObject(cls, data: bytes, device=None) -> "Quantizer":
        """Quantizer.readObject (Quantizer.java:205-226)."""
        if len(data) < 8:
            raise SketchMLException("truncated Quantizer stream")
        B, n = struct.unpack(">ii", data[:8])
        q = (QuantileQuantizer if cls is Quantizer else cls)(B)
        q.device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        q.n = n
        nbytes = _lib.lib.skml_dense_payload_bytes(n, B)
        if nbytes == 0:
            raise SketchMLException(f"bad Quantizer stream binNum={B} n={n}")
        q.payload = alloc_aligned(nbytes, q.device)
        arr = np.frombuffer(data, dtype=np.uint8).copy()
        check(_lib.lib.skml_dense_deserialize_ref(q._ctx().handle, arr.ctypes.data_as(_lib.u8p), len(arr),
                                                  C.c_void_p(q.payload.data_ptr()), nbytes), "readObject")
        q._load_header()
        return q


class QuantileQuantizer(Quantizer):
    """quantization/QuantileQuantizer.java:18-99 on the GPU.

    `seed` seeds the java.util.Random stream that the reference draws from its JVM-global
    Random (QSketchUtils.java:9): same seed -> same splits and bins as the oracle.
    """

    def __init__(self, binNum: int = Quantizer.DEFAULT_BIN_NUM, seed: int = 0, deferred: bool = False):
        super().__init__(binNum, seed, deferred)

    def quantize(self, values) -> None:
        """QuantileQuantizer.quantize (QuantileQuantizer.java:27-50)."""
        self._encode(values, dedup=True)

    def parallelQuantize(self, values) -> None:
        """QuantileQuantizer.parallelQuantize (QuantileQuantizer.java:53-92): T =
        Constants.Parallel.getParallelism() slice sketches merged in slice order, and, as in the
        reference, no Maths.unique of the splits.  The compaction bits follow the schedule that
        runs the slices one after another, then the merges, from Random(seed)
        (skml_dense_encode_parallel_f32)."""
        self._encode(values, dedup=False, threads=Parallel.getParallelism())

    def quantizationType(self) -> QuantizationType:
        return QuantizationType.QUANTILE

    @classmethod
    def quantizeBuckets(cls, buckets, binNum: int = Quantizer.DEFAULT_BIN_NUM, seed: int = 0) -> list:
        """QuantileQuantizer.quantize of each of several independent buckets (e.g. the gradient
        buckets of one step), identical per bucket to quantize(); fp32 buckets are encoded by
        skml_dense_encode_batch_f32, which overlaps one bucket's sketch with the previous
        bucket's quantize pass on two streams."""
        xs = [as_device_values(b) for b in buckets]
        qs = [cls(binNum, seed) for _ in xs]
        if not xs:
            return qs
        if any(x.dtype != torch.float32 for x in xs) or len({x.device for x in xs}) != 1:
            for q, x in zip(qs, xs):
                q.quantize(x)
            return qs
        p = _lib.Params()
        _lib.lib.skml_params_default(C.byref(p))
        p.bin_num = int(binNum)
        p.seed = int(seed)
        p.dedup = 1
        nb = len(xs)
        ptrs = (C.c_void_p * nb)()
        pls = (C.c_void_p * nb)()
        ns = np.zeros(nb, dtype=np.int64)
        caps = (C.c_size_t * nb)()
        for i, (q, x) in enumerate(zip(qs, xs)):
            q.device, q.n, q._wide = x.device, x.numel(), False
            cap = _lib.lib.skml_dense_payload_bytes(q.n, q.binNum)
            if cap == 0:
                raise SketchMLException(f"bad quantizer arguments n={q.n} binNum={q.binNum}")
            q.payload = alloc_aligned(cap, x.device)
            ptrs[i], pls[i], ns[i], caps[i] = x.data_ptr(), q.payload.data_ptr(), q.n, cap
        st = _lib.lib.skml_dense_encode_batch_f32(qs[0]._ctx().handle, nb, ptrs, ns.ctypes.data_as(_lib.i64p),
                                                  C.byref(p), pls, caps)
        check(st, "quantize")
        for q in qs:
            q._load_header()  # synchronises; surfaces NaN as QuantileSketchException
        return qs


class UniformQuantizer(Quantizer):
    """quantization/UniformQuantizer.java:14-76 on the GPU: bin_num equal-width bins between the
    Java min and max (MAX_VALUE / MIN_VALUE initialised), no Maths.unique, NaN values binned by
    indexOf rather than rejected."""

    def __init__(self, binNum: int = Quantizer.DEFAULT_BIN_NUM, seed: int = 0, deferred: bool = False):
        super().__init__(binNum, seed, deferred)

    def quantize(self, values) -> None:
        """UniformQuantizer.quantize (UniformQuantizer.java:21-45)."""
        self._encode(values, dedup=False, uniform=True)

    def parallelQuantize(self, values) -> None:
        """UniformQuantizer.parallelQuantize (UniformQuantizer.java:48-70): the same splits and
        bins as quantize (only the indexOf loop is sliced over threads in the reference)."""
        Parallel.getParallelism()  # parallelQuantizeToBins reads it (Quantizer.java:94-117)
        self._encode(values, dedup=False, uniform=True)

    def quantizationType(self) -> QuantizationType:
        return QuantizationType.UNIFORM


DEFAULT_BIN_NUM = Quantizer.DEFAULT_BIN_NUM

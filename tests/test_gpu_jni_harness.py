"""The JNI shim (jni/skml_jni.c) executed end to end on the GPU under a simulated JVM.

No JDK exists in this image, so the Java classes under jni/java/ cannot be compiled.  The C half of
the drop-in can still run: the shim is compiled here against jni/test/jni.h (the declaration-only
JNI 1.8 subset it uses) into a scratch directory, and this test provides the JNIEnv function table
from Python (ctypes callbacks): Java arrays are numpy arrays behind opaque handles,
GetPrimitiveArrayCritical hands out their memory, ThrowNew records the pending exception as the
JVM would.  Each native is then called exactly as HipCodec.java declares it, and its results are
checked against the oracle: QuantileQuantizer.quantize through encodeDenseF64 / info / getBins /
decodeDenseF64 (HipQuantileQuantizer), UniformQuantizer through encodeDenseUniformF64
(HipUniformQuantizer, HipDenseVectorCompressor(UNIFORM)), the sparse path through
encodeSparse / decodeSparse, DeltaAdaptive through deltaEncode, and the exception mapping
(NaN -> QuantileSketchException, HeapQuantileSketch.java:75-76)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PFX = "Java_org_dma_sketchml_hip_HipCodec_"


class FakeJVM:
    """JNINativeInterface_ of jni/test/jni.h, backed by Python objects."""

    def __init__(self):
        self.objs = {}
        self.next = 16
        self.pending = None
        vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
        EP = C.c_void_p  # JNIEnv*
        self.fns = [
            ("FindClass", C.CFUNCTYPE(vp, EP, C.c_char_p), self._find_class),
            ("ThrowNew", C.CFUNCTYPE(i32, EP, vp, C.c_char_p), self._throw_new),
            ("GetArrayLength", C.CFUNCTYPE(i32, EP, vp), lambda e, a: len(self.objs[a])),
            ("NewByteArray", C.CFUNCTYPE(vp, EP, i32), lambda e, n: self.new(np.zeros(n, np.int8))),
            ("NewIntArray", C.CFUNCTYPE(vp, EP, i32), lambda e, n: self.new(np.zeros(n, np.int32))),
            ("NewLongArray", C.CFUNCTYPE(vp, EP, i32), lambda e, n: self.new(np.zeros(n, np.int64))),
            ("NewDoubleArray", C.CFUNCTYPE(vp, EP, i32), lambda e, n: self.new(np.zeros(n, np.float64))),
            ("SetByteArrayRegion", C.CFUNCTYPE(None, EP, vp, i32, i32, vp), self._set_region),
            ("SetLongArrayRegion", C.CFUNCTYPE(None, EP, vp, i32, i32, vp), self._set_region),
            ("SetDoubleArrayRegion", C.CFUNCTYPE(None, EP, vp, i32, i32, vp), self._set_region),
            ("GetPrimitiveArrayCritical", C.CFUNCTYPE(vp, EP, vp, vp), lambda e, a, c: self.objs[a].ctypes.data),
            ("ReleasePrimitiveArrayCritical", C.CFUNCTYPE(None, EP, vp, vp, i32), lambda e, a, p, m: None),
            ("ExceptionCheck", C.CFUNCTYPE(C.c_uint8, EP), lambda e: 1 if self.pending else 0),
        ]

        class Table(C.Structure):
            _fields_ = [(name, proto) for name, proto, _ in self.fns]

        self._cbs = [proto(fn) for _, proto, fn in self.fns]  # keep the callbacks alive
        self.table = Table(*self._cbs)
        self.table_ptr = C.pointer(self.table)
        self._envp = C.pointer(C.c_void_p(C.cast(self.table_ptr, C.c_void_p).value))
        self.env = C.cast(self._envp, C.c_void_p)  # JNIEnv*: a pointer to the table pointer

    def new(self, arr):
        h = self.next
        self.next += 16
        self.objs[h] = arr
        return h

    def _find_class(self, env, name):
        return self.new(np.frombuffer(name, dtype=np.uint8).copy())

    def _throw_new(self, env, cls, msg):
        self.pending = (bytes(self.objs[cls]).decode(), (msg or b"").decode())
        return 0

    def _set_region(self, env, arr, start, n, buf):
        a = self.objs[arr]
        if n:
            C.memmove(a.ctypes.data + start * a.itemsize, buf, n * a.itemsize)

    def take_exception(self):
        e, self.pending = self.pending, None
        return e


@pytest.fixture(scope="module")
def jni(tmp_path_factory):
    out = tmp_path_factory.mktemp("jni") / "libskml_jni_test.so"
    lib = os.path.join(ROOT, "sketchml_amd", "lib")
    r = subprocess.run(["gcc", "-std=c11", "-O1", "-shared", "-fPIC", "-I", os.path.join(ROOT, "jni", "test"),
                        "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "jni", "skml_jni.c"), "-L", lib,
                        "-lskml", "-Wl,-rpath," + lib, "-o", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    import sketchml_amd  # noqa: F401  (torch and libskml.so first, as in every GPU test)
    L = C.CDLL(str(out))
    vm = FakeJVM()
    ctx = _proto(L, "ctxCreate", C.c_int64, [C.c_int32])(vm.env, None, 0)
    assert ctx and vm.pending is None
    yield L, vm, ctx
    _proto(L, "ctxDestroy", None, [C.c_int64])
    getattr(L, PFX + "ctxDestroy")(vm.env, None, ctx)


def _proto(L, name, res, args):
    f = getattr(L, PFX + name)
    f.restype = res
    f.argtypes = [C.c_void_p, C.c_void_p] + args
    return f


def _info(L, vm, payload):
    h = _proto(L, "info", C.c_void_p, [C.c_void_p])(vm.env, None, payload)
    return vm.objs[h]


def test_jni_quantile_dense_roundtrip(jni):
    """HipQuantileQuantizer.quantize / HipDenseVectorCompressor(QUANTILE): encodeDenseF64 (with
    Maths.unique), info, getBins and decodeDenseF64 against QuantileQuantizer.quantize."""
    L, vm, ctx = jni
    x = np.random.default_rng(21).standard_normal(300007)
    hx = vm.new(x)
    enc = _proto(L, "encodeDenseF64", C.c_void_p, [C.c_int64, C.c_void_p, C.c_int32, C.c_uint8, C.c_int64, C.c_int32])
    pl = enc(vm.env, None, ctx, hx, 256, 1, 11, 1)
    assert pl and vm.pending is None
    oq = O.quantize(x, 256, 11)
    info = _info(L, vm, pl)
    assert (int(info[0]), int(info[1]), int(info[2]), info[3], info[4]) == (oq.bin_num, len(x), oq.zero_idx, oq.min,
                                                                              oq.max)
    assert np.array_equal(info[5: 5 + oq.bin_num - 1], oq.splits)
    bins = vm.new(np.zeros(len(x), np.int32))
    _proto(L, "getBins", None, [C.c_void_p, C.c_void_p])(vm.env, None, pl, bins)
    assert np.array_equal(vm.objs[bins], oq.bins)
    out = vm.new(np.zeros(len(x), np.float64))
    _proto(L, "decodeDenseF64", None, [C.c_int64, C.c_void_p, C.c_void_p])(vm.env, None, ctx, pl, out)
    assert vm.pending is None
    assert np.array_equal(vm.objs[out], oq.values()[oq.bins])


def test_jni_uniform_dense(jni):
    """HipUniformQuantizer / HipDenseVectorCompressor(UNIFORM): encodeDenseUniformF64 against
    UniformQuantizer.quantize (quantization/UniformQuantizer.java:21-45)."""
    L, vm, ctx = jni
    x = np.random.default_rng(22).standard_normal(123457) * 3.0
    pl = _proto(L, "encodeDenseUniformF64", C.c_void_p, [C.c_int64, C.c_void_p, C.c_int32])(vm.env, None, ctx,
                                                                                            vm.new(x), 64)
    assert pl and vm.pending is None
    oq = O.uniform_quantize(x, 64)
    info = _info(L, vm, pl)
    assert (int(info[0]), int(info[2]), info[3], info[4]) == (oq.bin_num, oq.zero_idx, oq.min, oq.max)
    assert np.array_equal(info[5: 5 + oq.bin_num - 1], oq.splits)
    bins = vm.new(np.zeros(len(x), np.int32))
    _proto(L, "getBins", None, [C.c_void_p, C.c_void_p])(vm.env, None, pl, bins)
    assert np.array_equal(vm.objs[bins], oq.bins)


def test_jni_nan_raises_quantile_sketch_exception(jni):
    L, vm, ctx = jni
    x = np.random.default_rng(23).standard_normal(5000)
    x[77] = np.nan
    enc = _proto(L, "encodeDenseF64", C.c_void_p, [C.c_int64, C.c_void_p, C.c_int32, C.c_uint8, C.c_int64, C.c_int32])
    assert not enc(vm.env, None, ctx, vm.new(x), 256, 1, 1, 1)
    cls, msg = vm.take_exception()
    assert cls == "org/dma/sketchml/sketch/sketch/quantile/QuantileSketchException" and msg == "Encounter NaN value"


def test_jni_sparse_roundtrip(jni):
    """HipSparseVectorCompressor.compressSparse / decompressSparse: encodeSparse + decodeSparse
    against SparseVectorCompressor's quantize + GroupedMinMaxSketch (values as quantValues[bin])."""
    L, vm, ctx = jni
    rng = np.random.default_rng(24)
    keys = np.nonzero(rng.random(200000) < 0.2)[0].astype(np.int32)
    vals = rng.standard_normal(len(keys))
    enc = _proto(L, "encodeSparse", C.c_int64, [C.c_int64, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                                 C.c_double, C.c_int64, C.c_int64, C.c_uint8, C.c_int32])
    sp = enc(vm.env, None, ctx, vm.new(keys), vm.new(vals), 256, 8, 2, 0.3, 5, 6, 0, 1)
    assert sp and vm.pending is None
    nnz = _proto(L, "sparseNnz", C.c_int32, [C.c_int64])(vm.env, None, sp)
    assert nnz == len(keys)
    ko, vo = vm.new(np.zeros(nnz, np.int32)), vm.new(np.zeros(nnz, np.float64))
    _proto(L, "decodeSparse", None, [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p])(vm.env, None, ctx, sp, ko, vo)
    assert vm.pending is None
    _proto(L, "freeSparse", None, [C.c_int64])(vm.env, None, sp)
    osp = O.sparse_compress(keys, vals, 256, 8, 2, 0.3, 5, 6)
    ok, ob = osp.restore()
    assert np.array_equal(vm.objs[ko], ok)
    assert np.array_equal(vm.objs[vo], osp.q.values()[ob])


def test_jni_delta_encode(jni):
    """HipDeltaAdaptiveEncoder.encode: deltaEncode's {numIntervals, flagKind, bit lengths, word
    counts, words...} against DeltaAdaptiveEncoder.encode (binary/DeltaAdaptiveEncoder.java:54-112)."""
    L, vm, ctx = jni
    keys = np.cumsum(np.random.default_rng(25).integers(1, 40, 50000)).astype(np.int32)
    h = _proto(L, "deltaEncode", C.c_void_p, [C.c_int64, C.c_void_p])(vm.env, None, ctx, vm.new(keys))
    assert h and vm.pending is None
    r = vm.objs[h]
    want = O.delta_encode(keys)
    assert (int(r[0]), int(r[1]), int(r[2]), int(r[3])) == (want["num_intervals"], int(want["flag_kind"]),
                                                          want["n_flag_bits"], want["n_delta_bits"])
    nf, nd = int(r[4]), int(r[5])
    assert (nf, nd) == (len(want["flag_words"]), len(want["delta_words"]))
    assert np.array_equal(r[6: 6 + nf].astype(np.uint64), want["flag_words"][:nf])
    assert np.array_equal(r[6 + nf: 6 + nf + nd].astype(np.uint64), want["delta_words"][:nd])

#!/usr/bin/env python3
"""Sparse-path measurement (BASELINE config 3): a 2^28-dim dense fp32 gradient with 10 % nnz,
DenseDoubleGradient.toSparse -> SparseVectorCompressor.compressSparse -> decompressSparse.

Prints one JSON line: per-phase device times (HIP events on the codec stream), dense-input
throughput, and the algorithmic-byte roofline of SURVEY.md §8(d) (sparse encode ~ 6.2 B per
dense element at rho = 0.1: 4 dense read + rho*(8 write kv + 4 sketch re-read + 8 partition
re-read + ~2 payload)).

usage: python tools/bench_sparse.py [--dim 268435456] [--density 0.1] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=2**28)
    ap.add_argument("--density", type=float, default=0.1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--aggregate", type=int, default=0,
                    help="also time Gradient.sum of this many payloads (skml_sparse_decode_sum_f64)")
    ap.add_argument("--only-e2e", action="store_true",
                    help="one warm-up and `reps` timed dense -> payload encodes only (the PMC passes' program)")
    ap.add_argument("--only-decode", action="store_true",
                    help="one encode, then one warm-up and `reps` timed restores (decompressSparse) only")
    a = ap.parse_args()
    import sketchml_amd as sk
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import forms  # noqa: E402
    forms.apply()  # SKML_TOOL_FORMS (tools/ab.sh)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(a.dim, device=dev, generator=g)
    x[torch.rand(a.dim, device=dev, generator=g) >= a.density] = 0.0
    torch.cuda.synchronize()

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps, out

    if a.only_decode:
        pl0 = sk.encode_dense_as_sparse(x, 256, 8, 2, 0.3, 3, 3)
        t_dec, _ = timed(lambda: pl0.restore(), a.reps)
        print(json.dumps({"decode_ms": round(t_dec * 1e3, 3)}))
        return
    if a.only_e2e:
        t_e2e, _ = timed(lambda: sk.encode_dense_as_sparse(x, 256, 8, 2, 0.3, 3, 3), a.reps)
        print(json.dumps({"dense_to_payload_ms": round(t_e2e * 1e3, 3)}))
        return
    t_compact, (keys, vals) = timed(lambda: sk.to_sparse(x), a.reps)
    nnz = keys.numel()
    t_encode, pl = timed(lambda: sk.encode_sparse(keys, vals, 256, 8, 2, 0.3, 3, 3), a.reps)
    t_e2e, pl2 = timed(lambda: sk.encode_dense_as_sparse(x, 256, 8, 2, 0.3, 3, 3), a.reps)
    t_decode, (rk, rv) = timed(lambda: pl.restore(), a.reps)
    ok = bool(torch.equal(rk, keys))
    import ctypes as C
    import numpy as np
    from sketchml_amd import _lib
    from sketchml_amd.context import get_context
    ctx = get_context(0).handle
    warm = np.empty(pl2.export_bytes() * 2, dtype=np.uint8)  # first use of the wire kernels, untimed
    pl2.serialize()
    fresh = sk.encode_sparse(keys, vals, 256, 8, 2, 0.3, 3, 3)
    torch.cuda.synchronize()
    del warm
    need = C.c_size_t()
    # the destination is a resident byte array, as a JVM byte[] is (allocated zeroed): a fresh
    # np.empty's first-touch page faults would otherwise be timed as part of the copy
    buf = np.zeros(pl2.export_bytes(), dtype=np.uint8)
    buf.fill(1)
    t0 = time.perf_counter()
    # the C entry points themselves (the JNI path: one call into a byte[]), first call = build
    assert _lib.lib.skml_sparse_serialize(ctx, fresh.handle, None, 0, C.byref(need)) == 0
    assert need.value <= len(buf)
    assert _lib.lib.skml_sparse_serialize(ctx, fresh.handle, buf.ctypes.data_as(_lib.u8p), need.value, C.byref(need)) == 0
    t_ser = time.perf_counter() - t0
    buf = buf[: need.value]
    t0 = time.perf_counter()
    assert _lib.lib.skml_sparse_serialize(ctx, fresh.handle, buf.ctypes.data_as(_lib.u8p), need.value, C.byref(need)) == 0
    t_ser_copy = time.perf_counter() - t0
    stream = buf.tobytes()
    qv = pl.values()

    def read():
        h = C.c_void_p()
        assert _lib.lib.skml_sparse_deserialize(ctx, buf.ctypes.data_as(_lib.u8p), len(buf), qv.ctypes.data_as(_lib.dblp),
                                                len(qv), C.byref(h)) == 0, _lib.last_error()
        return sk.SparsePayload(h, 0, 2)
    t_read, back = timed(read, a.reps)
    bk, bv = back.restore()
    read_ok = bool(torch.equal(bk, keys)) and bool(torch.equal(bv, rv))
    rho = nnz / a.dim
    alg = (4.0 + rho * (8 + 4 + 8 + 2)) * a.dim
    line = {
        "metric": "sparse grad encode GB/s (fp32 dense in), C3",
        "value": round(4.0 * a.dim / t_e2e / 1e9, 2), "unit": "GB/s",
        "config": {"workload": f"C3: {a.dim}-dim dense fp32, {a.density:.0%} nnz (Bernoulli), 256 bins, "
                               "8 groups, 2 rows, colRatio 0.3", "nnz": nnz},
        "ms": {"compact": round(t_compact * 1e3, 3), "encode_kv": round(t_encode * 1e3, 3),
               "dense_to_payload": round(t_e2e * 1e3, 3), "decode": round(t_decode * 1e3, 3),
               "write_object": round(t_ser * 1e3, 3), "write_object_cached_copy": round(t_ser_copy * 1e3, 3),
               "read_object": round(t_read * 1e3, 3)},
        "stream_bytes": len(stream), "read_object_roundtrip_exact": read_ok,
        "roofline": {"bound": "hbm", "alg_bytes": alg, "achieved_gbs": round(alg / t_e2e / 1e9, 1),
                     "peak": HBM, "frac": round(alg / t_e2e / 1e9 / HBM, 4)},
        "compact_gbs": round((4.0 * a.dim + 8.0 * nnz) / t_compact / 1e9, 1),
        "keys_roundtrip_exact": ok,
        "note": "wall time of synchronising calls (the encode plans on the device and reads the "
                "quantizer header and group table back once; dense_to_payload adds the compaction's nnz read-back)",
    }
    if a.aggregate:
        from sketchml_amd.distributed import blob_stride
        # distinct payloads, as in the DP step: rank r's C3 gradient (dense seed 3 + r), bench.py's data
        pls = [pl2]
        for r in range(1, a.aggregate):
            gr = torch.Generator(device=dev).manual_seed(3 + r)
            xr = torch.randn(a.dim, device=dev, generator=gr)
            xr[torch.rand(a.dim, device=dev, generator=gr) >= a.density] = 0.0
            pls.append(sk.encode_dense_as_sparse(xr, 256, 8, 2, 0.3, 3 + r, 3 + r))
            del xr
        stride = blob_stride([p.export_bytes() for p in pls])
        allb = torch.zeros(stride * len(pls), dtype=torch.uint8, device=dev)
        for i, p in enumerate(pls):
            p.export(allb[i * stride:(i + 1) * stride])
        del pls
        t_sum, _ = timed(lambda: sk.decode_sum(allb, a.aggregate, stride, a.dim, 1.0 / a.aggregate), a.reps)
        line["ms"]["decode_sum"] = round(t_sum * 1e3, 3)
        line["aggregate"] = {"payloads": a.aggregate, "blob_stride": stride, "distinct": True}
    print(json.dumps(line))


if __name__ == "__main__":
    main()

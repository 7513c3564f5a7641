#!/usr/bin/env python3
"""Probe: throughput of independent bucket encodes issued on two HIP streams with two codec
contexts (each its own workspace), against one stream.  Buckets alternate A/B, so bucket i+1's
VALU-bound leaf can run beside bucket i's HBM-bound quantize."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

L = _lib.lib
n, steps, nbuf = 2**26, 200, 4
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
xs = []
for b in range(nbuf):
    g.manual_seed(4 + 1000 * b)
    xs.append(torch.randn(n, device=dev, generator=g))
nb = L.skml_dense_payload_bytes(n, 256)
pls = [sk.alloc_aligned(nb, dev) for _ in range(2)]
p = _lib.Params()
L.skml_params_default(C.byref(p))
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
ctxs = []
for s in streams:
    h = C.c_void_p()
    assert L.skml_ctx_create(0, C.c_void_p(s.cuda_stream), C.byref(h)) == 0
    ctxs.append(h)


def run(k):
    for i in range(steps):
        j = i % k
        with torch.cuda.stream(streams[j]):
            L.skml_dense_encode_f32(ctxs[j], C.c_void_p(xs[i % nbuf].data_ptr()), n, C.byref(p),
                                    C.c_void_p(pls[j].data_ptr()), nb)


for k in (1, 2, 1, 2):
    run(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"streams={k} ms_per_bucket={dt * 1e3:.4f} GB/s={4 * n / dt / 1e9:.1f}")

# the library's batch entry point (two internal lanes, offset by one sketch pass)
ctx = sk.get_context(0).handle
for nbk in (2, 4, 8, 16, 32):
    pls2 = [sk.alloc_aligned(nb, dev) for _ in range(nbk)]
    ptrs = (C.c_void_p * nbk)(*[xs[i % nbuf].data_ptr() for i in range(nbk)])
    pptr = (C.c_void_p * nbk)(*[q.data_ptr() for q in pls2])
    ns = (C.c_int64 * nbk)(*([n] * nbk))
    caps = (C.c_size_t * nbk)(*([nb] * nbk))
    reps = max(2, 64 // nbk)
    L.skml_dense_encode_batch_f32(ctx, nbk, ptrs, ns, C.byref(p), pptr, caps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        assert L.skml_dense_encode_batch_f32(ctx, nbk, ptrs, ns, C.byref(p), pptr, caps) == 0
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps / nbk
    print(f"batch nbk={nbk} ms_per_bucket={dt * 1e3:.4f} GB/s={4 * n / dt / 1e9:.1f}")
    del pls2

# two contexts on library-owned streams (SKML_STREAM_OWN), alternating, no fork/join
own = []
for _ in range(2):
    h = C.c_void_p()
    assert L.skml_ctx_create(0, C.c_void_p(-1), C.byref(h)) == 0
    own.append(h)
for rep in range(2):
    for i in range(steps):
        j = i % 2
        L.skml_dense_encode_f32(own[j], C.c_void_p(xs[i % nbuf].data_ptr()), n, C.byref(p),
                                C.c_void_p(pls[j].data_ptr()), nb)
    for h in own:
        L.skml_ctx_sync(h)
    t0 = time.perf_counter()
    for i in range(steps):
        j = i % 2
        L.skml_dense_encode_f32(own[j], C.c_void_p(xs[i % nbuf].data_ptr()), n, C.byref(p),
                                C.c_void_p(pls[j].data_ptr()), nb)
    for h in own:
        L.skml_ctx_sync(h)
    dt = (time.perf_counter() - t0) / steps
    print(f"own-stream contexts ms_per_bucket={dt * 1e3:.4f} GB/s={4 * n / dt / 1e9:.1f}")

# the batch entry point called from a non-default (non-null) stream
side = torch.cuda.Stream()
with torch.cuda.stream(side):
    ctx2 = sk.get_context(0).handle  # rebinds the context to `side`
    nbk = 32
    pls2 = [sk.alloc_aligned(nb, dev) for _ in range(nbk)]
    ptrs = (C.c_void_p * nbk)(*[xs[i % nbuf].data_ptr() for i in range(nbk)])
    pptr = (C.c_void_p * nbk)(*[q.data_ptr() for q in pls2])
    ns = (C.c_int64 * nbk)(*([n] * nbk))
    caps = (C.c_size_t * nbk)(*([nb] * nbk))
    L.skml_dense_encode_batch_f32(ctx2, nbk, ptrs, ns, C.byref(p), pptr, caps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        L.skml_dense_encode_batch_f32(ctx2, nbk, ptrs, ns, C.byref(p), pptr, caps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 2 / nbk
    print(f"batch from side stream ms_per_bucket={dt * 1e3:.4f} GB/s={4 * n / dt / 1e9:.1f}")

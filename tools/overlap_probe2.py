#!/usr/bin/env python3
"""Probe: do two library-owned streams overlap when created first (before any torch stream)?"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

L = _lib.lib
early = []
for _ in range(2):
    h = C.c_void_p()
    assert L.skml_ctx_create(0, C.c_void_p(-1), C.byref(h)) == 0
    early.append(h)
n, steps, nbuf = 2**26, 100, 4
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


def run(ctxs, label):
    for rep in range(2):
        t0 = time.perf_counter()
        for i in range(steps):
            j = i % len(ctxs)
            L.skml_dense_encode_f32(ctxs[j], C.c_void_p(xs[i % nbuf].data_ptr()), n, C.byref(p),
                                    C.c_void_p(pls[j].data_ptr()), nb)
        for h in ctxs:
            L.skml_ctx_sync(h)
        dt = (time.perf_counter() - t0) / steps
        print(f"{label} ms_per_bucket={dt * 1e3:.4f}")


run(early, "early-created pair")
late = []
for _ in range(2):
    h = C.c_void_p()
    assert L.skml_ctx_create(0, C.c_void_p(-1), C.byref(h)) == 0
    late.append(h)
run(late, "late-created pair")
run([early[0], late[0]], "early0+late0")
run([early[0], early[1], late[0], late[1]], "four")

"""Probe: per-step time of the dense encode issued eagerly vs replayed from a captured HIP graph."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

n = 2**26
dev = torch.device("cuda", 0)
xs = [torch.randn(n, device=dev) for _ in range(4)]
nb = _lib.lib.skml_dense_payload_bytes(n, 256)
pl = sk.alloc_aligned(nb, dev)
p = _lib.Params()
_lib.lib.skml_params_default(C.byref(p))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    ctx = sk.get_context(0).handle

    def step(i):
        assert _lib.lib.skml_dense_encode_f32(ctx, C.c_void_p(xs[i % 4].data_ptr()), n, C.byref(p),
                                              C.c_void_p(pl.data_ptr()), nb) == 0

    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(40):
        step(i)
    torch.cuda.synchronize()
    print("eager  us/step", (time.perf_counter() - t) / 40 * 1e6)
    graphs = []
    for b in range(4):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step(b)
        graphs.append(g)
    torch.cuda.synchronize()
    for i in range(5):
        graphs[i % 4].replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(40):
        graphs[i % 4].replay()
    torch.cuda.synchronize()
    print("graph  us/step", (time.perf_counter() - t) / 40 * 1e6)

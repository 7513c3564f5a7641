#!/usr/bin/env python3
"""Probe (profiling aid): skml_dense_encode_batch_f32 over P buckets of n floats, timed between
synchronisations, for kernel traces of how the two lanes' leaf and quantize passes overlap.

usage: python tools/batch_probe.py [--n 67108864] [--buckets 8] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import forms  # noqa: E402

forms.apply()  # SKML_TOOL_FORMS (tools/ab.sh)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2**26)
    ap.add_argument("--buckets", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    L = _lib.lib
    dev = torch.device("cuda", 0)
    ctx = sk.get_context(0).handle
    g = torch.Generator(device=dev)
    xs = []
    for b in range(a.buckets):
        g.manual_seed(4 + b)
        xs.append(torch.randn(a.n, device=dev, generator=g))
    nb = L.skml_dense_payload_bytes(a.n, 256)
    pls = [sk.alloc_aligned(nb, dev) for _ in range(a.buckets)]
    p = _lib.Params()
    L.skml_params_default(C.byref(p))
    P = a.buckets
    ptrs = (C.c_void_p * P)(*[x.data_ptr() for x in xs])
    pptr = (C.c_void_p * P)(*[q.data_ptr() for q in pls])
    ns = (C.c_int64 * P)(*([a.n] * P))
    caps = (C.c_size_t * P)(*([nb] * P))

    def run():
        if L.skml_dense_encode_batch_f32(ctx, P, ptrs, ns, C.byref(p), pptr, caps):
            raise RuntimeError(_lib.last_error())

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    print(json.dumps({"n": a.n, "buckets": P, "ms_per_call": round(t * 1e3, 4),
                      "ms_per_bucket": round(t / P * 1e3, 4), "gbps": round(4.0 * a.n * P / t / 1e9, 1)}))


if __name__ == "__main__":
    main()

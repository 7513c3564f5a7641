#!/usr/bin/env python3
"""C4's consumer alone: P dense payloads of n codes (batch-encoded from N(0,1) buckets seeded
4 + r) -> skml_dense_decode_sum_f32 (Gradient.sum in double + x 1/P -> fp32), HIP-event timed on
the codec stream.  Prints one JSON line with the kernel's mean time, GB/s of algorithmic bytes
(P * n * b / 8 codes read + 4 n fp32 written) and the fraction of the 8 TB/s roofline.  Under
rocprofv3 --pmc it is the short program the counter passes run (tools/pmc_decode_sum.sh).

usage: python tools/bench_decode_sum.py [--n 67108864] [--P 8] [--bins 256] [--reps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2**26)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--bins", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import sketchml_amd as sk
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import forms  # noqa: E402
    forms.apply()  # SKML_TOOL_FORMS (tools/ab.sh)
    from sketchml_amd import _lib
    lib = _lib.lib
    dev = torch.device("cuda", 0)
    ctx = sk.get_context(0).handle
    n, P = a.n, a.P
    xs = []
    for r in range(P):
        g = torch.Generator(device=dev).manual_seed(4 + r)
        xs.append(torch.randn(n, device=dev, generator=g))
    nb = lib.skml_dense_payload_bytes(n, a.bins)
    stride = (nb + 255) // 256 * 256
    allp = sk.alloc_aligned(stride * P, dev)
    p = _lib.Params()
    lib.skml_params_default(C.byref(p))
    p.bin_num, p.seed = a.bins, 4
    ptrs = (C.c_void_p * P)(*[x.data_ptr() for x in xs])
    pptr = (C.c_void_p * P)(*[allp.data_ptr() + i * stride for i in range(P)])
    ns = (C.c_int64 * P)(*([n] * P))
    caps = (C.c_size_t * P)(*([stride] * P))
    if lib.skml_dense_encode_batch_f32(ctx, P, ptrs, ns, C.byref(p), pptr, caps):
        raise RuntimeError(_lib.last_error())
    del xs
    out = torch.empty(n, dtype=torch.float32, device=dev)

    def run():
        st = lib.skml_dense_decode_sum_f32(ctx, C.c_void_p(allp.data_ptr()), P, stride, C.c_void_p(out.data_ptr()),
                                           n, 1.0 / P)
        if st:
            raise RuntimeError(_lib.last_error())

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    lib.skml_ctx_set_timing(ctx, 1 << 5)
    lib.skml_ctx_reset_stats(ctx)
    for _ in range(a.reps):
        run()
    cnt, ms = C.c_int64(), C.c_double()
    lib.skml_ctx_kernel_stats(ctx, 5, C.byref(cnt), C.byref(ms))
    lib.skml_ctx_set_timing(ctx, 0)
    hdr = _lib.DenseHeader()
    lib.skml_dense_info(ctx, C.c_void_p(allp.data_ptr()), C.byref(hdr), None, 0)
    us = 1000.0 * ms.value / max(cnt.value, 1)
    alg = P * n * hdr.code_bits / 8.0 + 4.0 * n
    print(json.dumps({"workload": f"{P} dense payloads of {n} codes ({hdr.code_bits}-bit, {hdr.bin_num} bins) -> "
                                  f"one fp32 sum x 1/{P}", "k_decode_sum_us": round(us, 2), "launches": cnt.value,
                      "alg_bytes": alg, "gbps": round(alg / (us * 1e-6) / 1e9, 1),
                      "roofline_frac": round(alg / (us * 1e-6) / 1e9 / 8000.0, 4)}))


if __name__ == "__main__":
    main()

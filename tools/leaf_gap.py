#!/usr/bin/env python3
"""Where the headline's per-step time goes outside the kernels, and why the leaf measured inside
bench.py's timed region differs from the untimed breakdown pass.

Runs the north-star encode (2^28 floats, 2 rotating 1 GiB buckets, seed 6) in alternating
blocks of `--steps` encodes: clean (no events), leaf-only events (round 4's timed region), all
kernels evented (the breakdown pass), and one synchronisation per step.  Prints one JSON line
per block and a summary.

usage: python tools/leaf_gap.py [--steps 20] [--reps 3] [--n 268435456]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=2**28)
    a = ap.parse_args()
    import sketchml_amd as sk
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import forms  # noqa: E402
    forms.apply()  # SKML_TOOL_FORMS (tools/ab.sh)
    from sketchml_amd import _lib
    lib = _lib.lib
    dev = torch.device("cuda", 0)
    ctx = sk.get_context(0).handle
    n = a.n
    gen = torch.Generator(device=dev)
    xs = []
    for b in range(2):
        gen.manual_seed(6 + 1000 * b)
        xs.append(torch.randn(n, device=dev, generator=gen))
    nb = lib.skml_dense_payload_bytes(n, 256)
    pl = sk.alloc_aligned(nb, dev)
    p = _lib.Params()
    lib.skml_params_default(C.byref(p))
    p.bin_num = 256
    p.seed = 6
    step_i = [0]

    def step():
        x = xs[step_i[0] % 2]
        step_i[0] += 1
        if lib.skml_dense_encode_f32(ctx, C.c_void_p(x.data_ptr()), n, C.byref(p), C.c_void_p(pl.data_ptr()), nb):
            raise RuntimeError(_lib.last_error())

    def stats():
        out = {}
        for kid, name in ((0, "leaf"), (1, "merge"), (3, "quantize")):
            cnt, ms = C.c_int64(), C.c_double()
            lib.skml_ctx_kernel_stats(ctx, kid, C.byref(cnt), C.byref(ms))
            if cnt.value:
                out[name] = round(1000.0 * ms.value / cnt.value, 2)
        return out

    def block(mode):
        mask = {"clean": 0, "leaf_events": 1, "all_events": -1, "sync_each": 0}[mode]
        torch.cuda.synchronize()
        lib.skml_ctx_set_timing(ctx, mask)
        lib.skml_ctx_reset_stats(ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
            if mode == "sync_each":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / a.steps
        ks = stats() if mask else {}
        lib.skml_ctx_set_timing(ctx, 0)
        return {"mode": mode, "ms_per_step": round(t * 1e3, 4), "kernels_us": ks}

    for _ in range(5):
        step()
    rows = []
    for r in range(a.reps):
        for mode in ("clean", "leaf_events", "all_events", "sync_each"):
            row = block(mode)
            row["rep"] = r
            rows.append(row)
            print(json.dumps(row), flush=True)
    summ = {}
    for mode in ("clean", "leaf_events", "all_events", "sync_each"):
        ms = [r["ms_per_step"] for r in rows if r["mode"] == mode]
        summ[mode] = {"ms_per_step_min": min(ms), "ms_per_step_max": max(ms)}
        lv = [r["kernels_us"].get("leaf") for r in rows if r["mode"] == mode and r["kernels_us"].get("leaf")]
        if lv:
            summ[mode]["leaf_us"] = lv
    print(json.dumps({"summary": summ}))


if __name__ == "__main__":
    main()

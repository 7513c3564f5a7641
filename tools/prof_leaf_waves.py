#!/usr/bin/env python3
"""Per-wave start/end spread of the leaf kernel (profiling build):

    make -C sketchml_amd/csrc OUT=../lib_prof EXTRA=-DSKML_PROF_LEAF
    SKML_LIB=sketchml_amd/lib_prof/libskml.so python tools/prof_leaf_waves.py [n]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import forms  # noqa: E402

forms.apply()  # SKML_TOOL_FORMS: e.g. leaf_split:1 (only one-wave-per-tile waves carry stamps)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2**26
tiles = min(65536, n // 256 // 64)
x = torch.randn(n, device="cuda")
q = sk.QuantileQuantizer(256, seed=1)
fn = _lib.lib.skml_debug_leafprof
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * (4 * tiles))()
for it in range(3):
    q.quantize(x)
    torch.cuda.synchronize()
    assert fn(buf, 4 * tiles) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) * 0.01
    en = (a[:, 1] - t0) * 0.01
    dur = en - st
    xcc = a[:, 3] & 0xF
    hw = a[:, 2]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    print(f"iter {it}: kernel span {en.max():.1f} us; start p50 {np.percentile(st, 50):.1f} max {st.max():.1f}; "
          f"dur min {dur.min():.1f} p50 {np.percentile(dur, 50):.1f} p90 {np.percentile(dur, 90):.1f} "
          f"max {dur.max():.1f}; end p10 {np.percentile(en, 10):.1f} p50 {np.percentile(en, 50):.1f} "
          f"p90 {np.percentile(en, 90):.1f}")
    if it == 2:
        for k in range(8):
            m = xcc == k
            if m.any():
                print(f"   xcc {k}: waves {m.sum()} dur p50 {np.percentile(dur[m], 50):.1f} max {dur[m].max():.1f} "
                      f"end max {en[m].max():.1f}")
        hist = np.histogram(dur, bins=10)
        print("   dur histogram:", list(hist[0]), [round(v, 1) for v in hist[1]])
        # resident waves over time (1 us steps): how much of the span the chip runs short of waves
        T = np.arange(0.0, en.max() + 1.0, 1.0)
        conc = np.searchsorted(np.sort(st), T, side="right") - np.searchsorted(np.sort(en), T, side="right")
        peak = conc.max()
        used = dur.sum() / (peak * en.max())
        t90 = T[np.nonzero(conc >= 0.9 * peak)[0][-1]]
        t50 = T[np.nonzero(conc >= 0.5 * peak)[0][-1]]
        # duration by start time (when in the kernel a wave starts decides whom it shares its SIMD with)
        order = np.argsort(st)
        for q in range(10):
            sel = order[q * len(order) // 10:(q + 1) * len(order) // 10]
            print(f"   start decile {q}: start {st[sel].min():6.1f}..{st[sel].max():6.1f} us  dur p10 "
                  f"{np.percentile(dur[sel], 10):6.1f} p50 {np.percentile(dur[sel], 50):6.1f} p90 {np.percentile(dur[sel], 90):6.1f}")
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez_compressed("gpurun_out/leaf_waves.npz", st=st, en=en, hw=hw, xcc=xcc)
        print(f"   resident waves: peak {peak}, wave-slot use over the span {used:.3f}; "
              f">= 90 % of peak until {t90:.0f} us, >= 50 % until {t50:.0f} us, span {en.max():.0f} us")

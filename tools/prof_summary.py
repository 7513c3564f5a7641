#!/usr/bin/env python3
"""Phase timing of the fused merge + summary workgroup (profiling build).

    make -C sketchml_amd/csrc OUT=../lib_prof EXTRA=-DSKML_PROF_SUMMARY
    SKML_LIB=sketchml_amd/lib_prof/libskml.so python tools/prof_summary.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2**26
x = torch.randn(n, device="cuda")
q = sk.QuantileQuantizer(256, seed=1)
names = ["merge start", "summary start", "setup", "min/max", "gather", "blocky rank", "prefix", "quantiles",
         "unique+zero", "lut start", "lut end"]
buf = (C.c_ulonglong * 32)()
for it in range(5):
    q.quantize(x)
    torch.cuda.synchronize()
    fn = _lib.lib.skml_debug_prof
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    assert fn(buf, 32) == 0
    t0 = buf[0]
    print("iter", it, " ".join(f"{names[k]}={(buf[k] - t0) * 0.01:.2f}us" for k in range(11)))

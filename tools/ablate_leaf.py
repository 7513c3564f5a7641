"""Profiling aid: time the truncated / occupancy variants of the sketch leaf kernel."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2**26
stages = [int(s) for s in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3]
x = torch.randn(n, device="cuda")
ctx = sk.get_context().handle
for stage in stages:
    ms = C.c_double()
    st = _lib.lib.skml_debug_leaf_stage(ctx, C.c_void_p(x.data_ptr()), n, stage, 20, C.byref(ms))
    assert st == 0, _lib.last_error()
    print(f"stage {stage:2d}: {ms.value * 1000:8.1f} us   ({4 * n / (ms.value * 1e-3) / 1e9:7.0f} GB/s)")

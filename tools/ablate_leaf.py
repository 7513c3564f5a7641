"""Profiling aid: time the truncated variants of the sketch leaf kernel (skml_debug_leaf_stage)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2**26
x = torch.randn(n, device="cuda")
ctx = sk.get_context().handle
res = {}
for stage in (0, 1, 2, 3):
    ms = C.c_double()
    st = _lib.lib.skml_debug_leaf_stage(ctx, C.c_void_p(x.data_ptr()), n, stage, 20, C.byref(ms))
    assert st == 0, _lib.last_error()
    res[stage] = ms.value * 1000
    print(f"stage {stage}: {res[stage]:8.1f} us   ({4 * n / (ms.value * 1e-3) / 1e9:7.0f} GB/s)")

#!/usr/bin/env python3
"""Phase timing of the upper merge + summary at 2^26 (profiling build, wall_clock64 stamps at
100 MHz).  Pass-1 workgroup 0: start / loaded / in-wave levels / cross-wave levels; the last
arriver: arrival, after its acquire; pass 2 the same four; then the summary phases.

    make -C sketchml_amd/csrc OUT=../lib_prof EXTRA=-DSKML_PROF_SUMMARY
    SKML_LIB=sketchml_amd/lib_prof/libskml.so python tools/prof_merge.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import sketchml_amd as sk  # noqa: E402
from sketchml_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2**26
x = torch.randn(n, device="cuda")
q = sk.QuantileQuantizer(256, seed=1)
slots = {"p1wg0_start": 12, "p1wg0_loaded": 13, "p1wg0_inwave": 14, "p1wg0_done": 15, "last_arrival": 20,
         "last_acquired": 21, "p2_start": 16, "p2_loaded": 17, "p2_bits": 22, "p2_l1": 23, "p2_l2": 24, "p2_l3": 25, "p2_inwave": 18, "p2_done": 19,
         "summary_start": 1, "setup": 2, "minmax": 3, "gather": 4, "blocky_rank": 5, "prefix": 6,
         "quantiles": 7, "unique_zero": 8, "lut_start": 9, "lut_hist": 30, "lut_scan": 31, "lut_end": 10, "warm_start": 26, "warm_end": 27}
buf = (C.c_ulonglong * 32)()
fn = _lib.lib.skml_debug_prof
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
rows = []
for it in range(8):
    q.quantize(x)
    torch.cuda.synchronize()
    assert fn(buf, 32) == 0
    t0 = buf[12]
    rows.append({k: round((buf[v] - t0) * 0.01, 2) for k, v in slots.items()})
for r in rows[3:]:
    print(json.dumps(r))
# shader clock over the LUT phase: s_memtime ticks (g_prof 28..29) / wall time (9..10)
print("lut clock GHz", (buf[29] - buf[28]) / max(1, (buf[10] - buf[9])) * 0.1)

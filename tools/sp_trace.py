#!/usr/bin/env python3
"""Timeline of the last dense->payload encode in a rocprofv3 kernel trace of tools/bench_sparse.py
(start offset, gap before, duration in us per kernel).  usage: sp_trace.py [trace.csv] [n]"""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_sp/run_kernel_trace.csv"
count = int(sys.argv[2]) if len(sys.argv) > 2 else 27
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
i0 = [i for i, r in enumerate(rows) if "k_compact" in r["Kernel_Name"]][-1]
t0 = pe = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + count]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1000:9.1f} gap {(s - pe) / 1000:7.1f} dur {(e - s) / 1000:8.1f}  {r['Kernel_Name'][:60]}")
    pe = e

#!/usr/bin/env python3
"""Kernel durations and the idle gaps between consecutive kernels from a rocprofv3
--kernel-trace CSV (Start_Timestamp / End_Timestamp in ns).  Groups the gaps by the pair of
kernels they separate.

usage: python tools/trace_gaps.py DIR_OR_CSV [--skip 10]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def short(name):
    return name.split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip", type=int, default=10, help="leading kernels to ignore (warm-up)")
    ap.add_argument("--timeline", type=int, default=0, help="also print the last N operations in order")
    a = ap.parse_args()
    paths = [a.path] if a.path.endswith(".csv") else glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                                 recursive=True)
    rows = []
    for p in paths:
        rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in csv.DictReader(open(p))]
    copies = []
    if not a.path.endswith(".csv"):
        for p in glob.glob(os.path.join(a.path, "**", "*memory_copy_trace.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                               "copy " + r.get("Direction", r.get("Operation", "?"))))
    rows.sort()
    if a.timeline:
        ops = sorted(rows + copies)[-a.timeline:]
        t0, prev = ops[0][0], ops[0][0]
        for s_, e_, k in ops:
            print(f"{(s_ - t0) / 1e3:10.1f} gap {(s_ - prev) / 1e3:8.1f} dur {(e_ - s_) / 1e3:8.1f}  {k}")
            prev = max(prev, e_)
    rows = [r for r in rows if r[2].startswith("k_")][a.skip:]
    dur, gap = {}, {}
    for i, (s, e, k) in enumerate(rows):
        dur.setdefault(k, []).append((e - s) / 1e3)
        if i:
            ps, pe, pk = rows[i - 1]
            gap.setdefault(f"{pk} -> {k}", []).append((s - pe) / 1e3)
    out = {"kernels_us": {k: {"n": len(v), "mean": round(statistics.mean(v), 2), "min": round(min(v), 2),
                              "max": round(max(v), 2)} for k, v in dur.items()},
           "gaps_us": {k: {"n": len(v), "mean": round(statistics.mean(v), 2), "median": round(statistics.median(v), 2)}
                       for k, v in gap.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Side-by-side per-kernel averages of rocprofv3 --stats runs: kstats_cmp.py DIR_A DIR_B [filter...]
(each DIR holds a *kernel_stats.csv somewhere below it).  Prints calls and mean us per kernel."""
import csv
import glob
import os
import sys


def load(d):
    out = {}
    for p in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Name"].split("(")[0].replace("void ", "")
            out[name] = (int(r["Calls"]), float(r["AverageNs"]) / 1000.0, float(r["TotalDurationNs"]) / 1000.0)
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
flt = sys.argv[3:]
names = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0, 0))[2], b.get(k, (0, 0, 0))[2]))
print(f"{'kernel':60s} {'A calls':>8s} {'A us':>9s} {'B calls':>8s} {'B us':>9s}")
for k in names:
    if flt and not any(f in k for f in flt):
        continue
    ca, ua, _ = a.get(k, (0, 0.0, 0))
    cb, ub, _ = b.get(k, (0, 0.0, 0))
    print(f"{k[:60]:60s} {ca:8d} {ua:9.1f} {cb:8d} {ub:9.1f}")

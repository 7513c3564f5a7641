#!/usr/bin/env python3
"""Merged timeline (kernels + memory copies) from a rocprofv3 rocpd database (the default output
of rocprofv3 --kernel-trace --memory-copy-trace in ROCm 7.2), and per-kernel stats.

usage: python tools/rocpd_timeline.py DB [--from NAME_SUBSTRING] [--count N] [--stats]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--from", dest="start", default=None, help="start at the n-th event whose name contains this")
    ap.add_argument("--nth", type=int, default=1)
    ap.add_argument("--count", type=int, default=80)
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    ev = [("K", n, s, e, None) for n, s, e in cur.execute("select name, start, end from kernels")]
    ev += [("M", n, s, e, z) for n, s, e, z in cur.execute("select name, start, end, size from memory_copies")]
    ev.sort(key=lambda t: t[2])
    if a.stats:
        agg = defaultdict(lambda: [0, 0.0])
        for k, n, s, e, _ in ev:
            key = (k, n.split("(")[0][:70])
            agg[key][0] += 1
            agg[key][1] += (e - s) / 1e3
        for (k, n), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{k} {c:6d} {t:12.1f} us  avg {t / c:10.2f}  {n}")
        return
    i0 = 0
    if a.start:
        hits = [i for i, t in enumerate(ev) if a.start in t[1]]
        i0 = hits[min(a.nth, len(hits)) - 1] if hits else 0
    t0 = ev[i0][2]
    prev_end = t0
    for k, n, s, e, z in ev[i0:i0 + a.count]:
        extra = f" {z / 1e6:.1f} MB" if z else ""
        print(f"{(s - t0) / 1e3:10.1f} gap {(s - prev_end) / 1e3:8.1f} dur {(e - s) / 1e3:8.1f} {k} {n.split('(')[0][:60]}{extra}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()

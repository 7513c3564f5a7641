#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes of `bench_sparse.py --only-e2e` (one timed
dense -> payload encode after one warm-up) into per-kernel HBM bytes of ONE encode.

Corrections as tools/pmc_summary.py (MI355X_MICROARCH.md, HBM section): read = 2 x FETCH_SIZE KiB
x 1024 on gfx950, write = WRITE_SIZE KiB x 1024.  The bench runs the encode twice (warm-up + 1
timed rep): each kernel's dispatches are split in two halves and the second half is summed, i.e.
the bytes one encode moves.  Algorithmic bytes: 4 B per dense element read plus
rho x (8 kv written + 4 values re-read by the sketch + 8 kv re-read by the partition + 2 payload)."""
import argparse
import csv
import glob
import json
import os
import re


def per_dispatch(d, counter):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
                if not m or "skml" not in r["Kernel_Name"]:
                    continue
                rows.append((int(r.get("Dispatch_Id", 0)), m.group(1), float(r["Counter_Value"])))
    rows.sort()
    return rows


def second_half(rows):
    by = {}
    for _, k, v in rows:
        by.setdefault(k, []).append(v)
    return {k: sum(v[len(v) // 2:]) for k, v in by.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--dim", type=int, default=2**28)
    ap.add_argument("--nnz", type=int, default=26844167)
    a = ap.parse_args()
    f = second_half(per_dispatch(a.fetch, "FETCH_SIZE"))
    w = second_half(per_dispatch(a.write, "WRITE_SIZE"))
    kernels = {}
    for k in sorted(set(f) | set(w)):
        rb = 2.0 * f.get(k, 0.0) * 1024.0
        wb = w.get(k, 0.0) * 1024.0
        kernels[k] = {"read_bytes": rb, "write_bytes": wb, "hbm_bytes": rb + wb}
    total = sum(v["hbm_bytes"] for v in kernels.values())
    rho = a.nnz / a.dim
    alg = (4.0 + rho * (8 + 4 + 8 + 2)) * a.dim
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tools/bench_sparse.py --only-e2e, C3",
           "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950), write = WRITE_SIZE KiB x 1024; one encode",
           "kernels": dict(sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes"])),
           "total_hbm_bytes": total, "alg_bytes": alg, "counter_to_alg_ratio": total / alg}
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps({"total_hbm_bytes": total, "alg_bytes": alg, "ratio": total / alg,
                      "top": {k: round(v["hbm_bytes"] / 1e6, 1) for k, v in list(out["kernels"].items())[:12]}}))


if __name__ == "__main__":
    main()

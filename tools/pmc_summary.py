#!/usr/bin/env python3
"""Fold two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of `bench.py` into
profiles/<name>_pmc.json, the per-launch HBM traffic that bench.py reports as roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950 FETCH_SIZE
tallies 128-B streaming requests at 64 B, so the read side is doubled; WRITE_SIZE is exact for
16-B/lane stores.  Per-launch values are medians over the dispatches of each kernel.

usage: pmc_summary.py --fetch DIR --write DIR --n N --out profiles/r01_pmc.json
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

# kernel symbol -> the name bench.py's per-kernel timers use
ALIAS = {"k_leaf2": "k_leaf", "k_leaf64": "k_leaf"}


def short_name(sym):
    m = re.search(r"(k_[A-Za-z0-9_]+)", sym)
    name = m.group(1) if m else sym
    return ALIAS.get(name, name)


def read_counter(d, counter):
    per = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = short_name(row["Kernel_Name"])
                if not k.startswith("k_"):  # library kernels only (skip torch / copy kernels)
                    continue
                per.setdefault(k, []).append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = read_counter(a.fetch, "FETCH_SIZE")
    write = read_counter(a.write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fk = statistics.median(fetch[k]) if k in fetch else None
        wk = statistics.median(write[k]) if k in write else None
        e = {"launches_sampled": max(len(fetch.get(k, [])), len(write.get(k, [])))}
        if fk is not None:
            e["fetch_size_kib_raw"] = fk
            e["read_bytes_per_launch"] = 2.0 * fk * 1024.0
        if wk is not None:
            e["write_size_kib_raw"] = wk
            e["write_bytes_per_launch"] = wk * 1024.0
        if fk is not None and wk is not None:
            e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
        kernels[k] = e
    out = {"n": a.n, "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py",
           "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950), write = WRITE_SIZE KiB x 1024",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

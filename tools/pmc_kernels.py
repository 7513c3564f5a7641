#!/usr/bin/env python3
"""Per-kernel mean of every counter in one or more rocprofv3 counter_collection CSVs (one JSON
object: kernel -> counter -> mean per dispatch, plus dispatch counts).
usage: pmc_kernels.py out.json run1/run_counter_collection.csv [run2/...]"""
import collections
import csv
import json
import sys

out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("skml::", "").replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: {"mean": sum(v) / len(v), "dispatches": len(v)} for c, v in d.items()} for k, d in acc.items()}
res["_units"] = "FETCH_SIZE / WRITE_SIZE in KB per dispatch (FETCH_SIZE reads 1/2 of streamed bytes on gfx950, "
res["_units"] += "see MI355X_MICROARCH.md); SQ_* per dispatch"
json.dump(res, open(out, "w"), indent=1, sort_keys=True)

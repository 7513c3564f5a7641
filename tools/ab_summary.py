#!/usr/bin/env python3
"""One summary line of an A/B run (tools/ab.sh): KIND NAME REP FILE."""
import json
import sys

kind, name, rep, path = sys.argv[1:5]
lines = [ln for ln in open(path).read().splitlines() if ln.startswith("{")]
d = json.loads(lines[-1])
if kind == "dense":
    out = {"ms_per_step": d["ms_per_step"], "kernels_us": {k: v["avg_us"] for k, v in d["extras"]["kernels"].items()}}
elif kind in ("sparse", "sparse_enc"):
    out = d.get("ms", d)
elif kind in ("gap", "gap26", "gap24"):
    out = d.get("summary", d)
else:
    out = d
print(name, rep, json.dumps(out))

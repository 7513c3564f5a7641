#!/bin/bash
# k_decode_sum at C4 (8 x 2^26 8-bit codes): time A/B of the bank-replicated tables (default) and
# the one-table-per-payload kernel (SKML_DECODE_SUM_PLAIN=1), then one LDS counter pass of each.
# usage (through gpurun): bash tools/pmc_decode_sum.sh TAG  -> gpurun_out/dsum_TAG/
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dsum_$TAG
mkdir -p "$OUT"
for i in 1 2 3; do
  SKML_DECODE_SUM_PLAIN=1 timeout -k 10 120 python3 tools/bench_decode_sum.py >> "$OUT/ab_plain.jsonl"
  timeout -k 10 120 python3 tools/bench_decode_sum.py >> "$OUT/ab_rep.jsonl"
done
tail -n 3 "$OUT/ab_plain.jsonl" "$OUT/ab_rep.jsonl"
SKML_DECODE_SUM_PLAIN=1 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU \
    -d "$OUT/pmc_plain" -o run --output-format csv -- python3 tools/bench_decode_sum.py --reps 5 > "$OUT/pmc_plain.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU \
    -d "$OUT/pmc_rep" -o run --output-format csv -- python3 tools/bench_decode_sum.py --reps 5 > "$OUT/pmc_rep.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, statistics
out = sys.argv[1]
res = {}
for tag in ("plain", "rep"):
    per = {}
    for p in glob.glob(os.path.join(out, "pmc_" + tag, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "decode_sum" in r["Kernel_Name"]:
                per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res[tag] = {c: statistics.mean(v) for c, v in per.items()}
json.dump({"source": "rocprofv3 --pmc (one pass per build), tools/bench_decode_sum.py, C4: 8 x 2^26 8-bit codes",
           "per_launch_mean": res}, open(os.path.join(out, "lds_counters.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
find "$OUT" -name "*counter_collection.csv" -size +20M -delete

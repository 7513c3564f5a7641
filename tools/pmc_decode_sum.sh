#!/bin/bash
# k_decode_sum at C4 (8 x 2^26 8-bit codes): time A/B of the occupancy kernel with and without the
# next step's code prefetch and the 16-element per-payload kernel (SKML_FORM_DECODE_SUM 1), then
# one LDS / VALU counter pass of each.  usage (through gpurun): bash tools/pmc_decode_sum.sh TAG
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dsum_$TAG
mkdir -p "$OUT"
VARIANTS="occ:SKML_TOOL_FORMS=decode_sum:0 occ_nopf:SKML_TOOL_FORMS=decode_sum:2 plain:SKML_TOOL_FORMS=decode_sum:1"
for i in 1 2 3; do
  for V in $VARIANTS; do
    env "${V#*:}" timeout -k 10 120 python3 tools/bench_decode_sum.py >> "$OUT/ab_${V%%:*}.jsonl"
  done
done
tail -n 3 "$OUT"/ab_*.jsonl
for V in $VARIANTS; do
  env "${V#*:}" timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
      -d "$OUT/pmc_${V%%:*}" -o run --output-format csv -- python3 tools/bench_decode_sum.py --reps 5 > "$OUT/pmc_${V%%:*}.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, statistics
out = sys.argv[1]
res = {}
for tag in ("occ", "occ_nopf", "plain"):
    per = {}
    for p in glob.glob(os.path.join(out, "pmc_" + tag, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if "decode_sum" in r["Kernel_Name"]:
                per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    res[tag] = {c: statistics.mean(v) for c, v in per.items()}
json.dump({"source": "rocprofv3 --pmc (one pass per variant), tools/bench_decode_sum.py, C4: 8 x 2^26 8-bit codes",
           "per_launch_mean": res}, open(os.path.join(out, "lds_counters.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
find "$OUT" -name "*counter_collection.csv" -size +20M -delete

#!/bin/bash
# Counters of the Gradient.sum kernels over tools/bench_sparse.py --aggregate 8 (8 distinct C3
# payloads): HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes), two SQ passes and the L2 requests.
# Forms from SKML_TOOL_FORMS (tools/forms.py), default none.
# usage (through gpurun): bash tools/pmc_agg.sh TAG  -> gpurun_out/pmc_agg_TAG/summary.json
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_agg_$TAG
mkdir -p "$OUT"
for PASS in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS" \
    "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY TCC_REQ_sum TCC_HIT_sum"; do
  NAME=$(echo $PASS | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $PASS --kernel-trace -d "$OUT/$NAME" -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --aggregate 8 > "$OUT/$NAME.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, re, statistics, sys
out = sys.argv[1]
res = {}
for p in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        if not m or not m.group(1).startswith(("k_agg", "k_dec_keys", "k_rs_merge")):
            continue
        res.setdefault(m.group(1), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summ = {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in res.items()}
for k, d in summ.items():
    if "FETCH_SIZE" in d: d["read_bytes (2 x FETCH_SIZE KiB, gfx950)"] = 2 * d["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in d: d["write_bytes"] = d["WRITE_SIZE"] * 1024
json.dump({"source": "rocprofv3 --pmc, tools/bench_sparse.py --reps 1 --aggregate 8; per dispatch means; forms: "
           + os.environ.get("SKML_TOOL_FORMS", "default"), "kernels": summ},
          open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(summ, indent=1))
PY
find "$OUT" -name "*counter_collection.csv" -size +20M -delete
find "$OUT" -name "*kernel_trace.csv" -size +20M -delete

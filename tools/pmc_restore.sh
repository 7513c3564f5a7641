#!/bin/bash
# Counters of the restore's kernels (tools/bench_sparse.py --only-decode, one C3 payload):
# instruction mix and wait cycles (two SQ passes), HBM bytes (FETCH_SIZE, WRITE_SIZE) and L2
# requests / hits.  usage (through gpurun): bash tools/pmc_restore.sh TAG -> gpurun_out/pmc_rs_TAG/summary.json
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_rs_$TAG
mkdir -p "$OUT"
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_REQ_sum TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $PASS -d "$OUT/p$i" -o run --output-format csv -- python3 tools/bench_sparse.py --only-decode --reps 3 > "$OUT/p$i.log" 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, re, statistics, sys
out = sys.argv[1]
res = {}
for p in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        if not m:
            continue
        res.setdefault(m.group(1), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
summ = {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in res.items()}
# the largest dispatch of each kernel (k_dec_keys runs twice per restore: the inner tiles and the
# few group-edge tiles, whose mean alone says little)
big = {k: {c: max(v) for c, v in d.items()} for k, d in res.items()}
for k, d in summ.items():
    if "FETCH_SIZE" in d: d["read_bytes (2 x FETCH_SIZE KiB, gfx950)"] = 2 * d["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in d: d["write_bytes"] = d["WRITE_SIZE"] * 1024
json.dump({"source": "rocprofv3 --pmc, tools/bench_sparse.py --only-decode --reps 3 (C3 restore); per dispatch means",
           "kernels": summ, "kernels_max_dispatch": big}, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k in ("k_dec_keys_p", "k_dec_keys", "k_rs_merge_pf", "k_dec_deltas", "k_dec_lens", "k_rs_bounds"):
    if k in summ:
        print(k, json.dumps({c: round(v) for c, v in big[k].items()}))
PY
find "$OUT" -name "*.csv" -size +20M -delete

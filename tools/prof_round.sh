#!/bin/bash
# Full profile set of bench.py's default run (GPU box): kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE passes (folded by pmc_summary.py), and one SQ counter pass.
# usage (through gpurun): bash tools/prof_round.sh TAG   -> gpurun_out/prof_TAG/{stats,pmc.json,sq.json}
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-configs --steps 20 > "$OUT/bench_under_rocprof.json" 2> "$OUT/stats.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 10 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 10 > "$OUT/write.log" 2>&1
python3 tools/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --n 268435456 --out "$OUT/pmc.json" > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    -d "$OUT/sq" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > "$OUT/sq.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, statistics
out = sys.argv[1]
per = {}
for p in glob.glob(os.path.join(out, "sq", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        if "skml" not in r["Kernel_Name"]:
            continue
        per.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
res = {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in per.items()}
json.dump({"source": "rocprofv3 --pmc SQ_* (one pass), bench.py --steps 5 (default: n=2^28)", "n": 268435456,
           "per_launch_mean": res},
          open(os.path.join(out, "sq.json"), "w"), indent=1)
PY
find "$OUT" -name "*counter_collection.csv" -size +20M -delete
find "$OUT" -name "*kernel_trace.csv" -size +20M -delete

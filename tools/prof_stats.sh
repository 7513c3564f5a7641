#!/bin/bash
# GPU-box profiling of bench.py: kernel-trace stats + two PMC passes (FETCH_SIZE, WRITE_SIZE).
# usage (through gpurun): bash tools/prof_stats.sh [tag]   -> gpurun_out/prof_<tag>/...
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 20 > "$OUT/stats.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 10 > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 10 > "$OUT/write.log" 2>&1
python3 tools/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --n 67108864 \
    --out "$OUT/pmc.json" > /dev/null
# keep only the small summaries (the traces are large)
find "$OUT" -name "*counter_collection.csv" -size +20M -delete
find "$OUT" -name "*kernel_trace.csv" -size +20M -delete

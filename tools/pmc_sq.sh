#!/bin/bash
# SQ counters of bench.py's kernels (one rocprofv3 --pmc pass; counters per pass <= 8 SQ slots)
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_sq
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    -d "$OUT/a" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > "$OUT/a.log" 2>&1

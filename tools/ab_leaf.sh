#!/bin/bash
# A/B of the dense encode between sketchml_amd/lib_old and sketchml_amd/lib (two alternating runs
# each), plus one SQ counter pass of the new build.  usage (through gpurun): bash tools/ab_leaf.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in $(seq ${REPS:-2}); do
for L in ${LIBS:-lib_old lib}; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-extras --no-configs > gpurun_out/ab_$L.log 2>&1
python -c "
import json,sys;d=json.loads(open('gpurun_out/ab_$L.log').read().strip().splitlines()[-1]);print('$L',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done
done
OUT=gpurun_out/prof_sq
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    -d "$OUT/a" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --no-configs --steps 5 --warmup 2 > "$OUT/a.log" 2>&1
python3 tools/pmc_kernels.py "$OUT/sq.json" $(find "$OUT/a" -name "*counter_collection.csv") && cat "$OUT/sq.json" | head -c 1500

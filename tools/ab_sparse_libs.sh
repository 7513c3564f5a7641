#!/bin/bash
# A/B of the C3 sparse encode between in-tree builds.  usage (through gpurun):
#   LIBS="lib lib_x" REPS=2 bash tools/ab_sparse_libs.sh
set -e
cd "$GRAFT_REPO_ROOT"
for i in $(seq ${REPS:-2}); do
for L in ${LIBS:-lib}; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 200 python tools/bench_sparse.py > gpurun_out/absp.json 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/absp.json'));print('$L',d['ms'])"
done
done

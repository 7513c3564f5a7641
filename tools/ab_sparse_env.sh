#!/bin/bash
# A/B of the sparse C3 path between environment settings of one build.
# usage (through gpurun): VARS="SKML_SP_FORK=delta SKML_SP_FORK=mm" REPS=3 bash tools/ab_sparse_env.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in $(seq ${REPS:-2}); do
for V in ${VARS}; do
env "$V" timeout -k 10 150 python tools/bench_sparse.py --reps 10 > gpurun_out/ab_sp_env.json 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/ab_sp_env.json').read().strip().splitlines()[-1]);print('$V',{k:d['ms'][k] for k in ('compact','encode_kv','dense_to_payload','decode')})" | tee -a gpurun_out/ab_sp_env.txt
done
done

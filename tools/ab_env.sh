#!/bin/bash
# A/B of the dense encode between environment settings of one build (e.g. kernel variants chosen
# by an environment switch).  usage (through gpurun): VARS="SKML_LEAF128=0 SKML_LEAF128=1" REPS=3 bash tools/ab_env.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for i in $(seq ${REPS:-2}); do
for V in ${VARS}; do
env "$V" timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-extras --no-configs > gpurun_out/abenv.log 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1]);print('$V',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done
done

#!/bin/bash
# A/B of the dense encode between in-tree library builds, alternating runs.
# usage (through gpurun): bash tools/ab_libs.sh ROUNDS N BUFFERS lib_a lib_b ...
set -e
cd "$GRAFT_REPO_ROOT"
R=$1; N=$2; B=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $R); do
for L in "$@"; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python bench.py --n $N --buffers $B --steps 100 --warmup 10 --no-cpu-baseline --no-extras --no-configs > gpurun_out/ab_$L.log 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/ab_$L.log').read().strip().splitlines()[-1]);print('$L $N',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done; done

#!/bin/bash
# Split (4 waves per tile) against one-wave-per-tile leaf across bucket sizes (SKML_LEAF_SPLIT).
# usage (through gpurun): bash tools/ab_leaf_split.sh
set -e
cd "$GRAFT_REPO_ROOT"
for N in 4194304 16777216 26844167 33554432 50331648 67108864; do
for V in 0 1; do
B=$(( N <= 33554432 ? 8 : 4 ))
SKML_LEAF_SPLIT=$V timeout -k 10 120 python bench.py --n $N --buffers $B --steps 200 --warmup 20 --no-cpu-baseline --no-extras --no-configs > gpurun_out/absplit.log 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/absplit.log').read().strip().splitlines()[-1]);print('N=$N split=$V',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done; done

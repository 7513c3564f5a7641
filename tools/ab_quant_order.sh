#!/bin/bash
# A/B of the dense encode at 2^26 and 2^28 between sketchml_amd/lib_old and sketchml_amd/lib (three
# alternating runs).  usage (through gpurun): bash tools/ab_quant_order.sh
set -e
cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
for L in lib_old lib; do
for N in 67108864 268435456; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python bench.py --n $N --buffers $([ $N = 67108864 ] && echo 4 || echo 1) --steps 100 --warmup 10 --no-cpu-baseline --no-extras --no-configs > gpurun_out/abq.log 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/abq.log').read().strip().splitlines()[-1]);print('$L $N',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done; done; done

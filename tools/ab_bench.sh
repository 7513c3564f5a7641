set -e
for i in 1 2; do
for L in lib_old lib; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab_$L.log 2>&1
python -c "
import json,sys;d=json.loads(open('gpurun_out/ab_$L.log').read().strip().splitlines()[-1]);print('$L',d['ms_per_step'],{k:v['avg_us'] for k,v in d['extras']['kernels'].items()})"
done
done

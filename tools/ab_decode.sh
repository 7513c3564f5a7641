set -e
mkdir -p gpurun_out/abd
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abd/tests.log 2>&1
for i in 1 2; do
for L in lib_old lib; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-configs > gpurun_out/abd/$L.$i.log 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/abd/$L.$i.log').read().strip().splitlines()[-1]);print('$L',d['ms_per_step'],d['extras']['kernels'].get('k_quantize'),d['extras']['decode']['avg_us'])"
done
done

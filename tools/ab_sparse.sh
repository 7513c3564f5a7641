for L in lib lib_c32768 lib_c65536; do
SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 120 python tools/bench_sparse.py --reps 5 > gpurun_out/sp_$L.json 2>&1
python -c "
import json;d=json.loads(open('gpurun_out/sp_$L.json').read().strip().splitlines()[-1]);print('$L',d['ms'])"
done

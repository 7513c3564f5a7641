# r04n: 16 keys per thread in the run-bounds kernels (k_agg_bounds, k_rs_bounds): parity and timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1
tail -1 gpurun_out/r04n_tests.log
for i in 1 2 3; do
  for V in pers:SKML_AB_DEFAULT=1 all:SKML_AGG_GRID_ALL=1; do
    env "${V#*:}" timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04n_${V%%:*}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04n_${V%%:*}_$i.json').read().strip().splitlines()[-1])
print('${V%%:*}', $i, {k: d['ms'][k] for k in ('encode_kv', 'dense_to_payload', 'decode', 'decode_sum')})"
  done
done
SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n_prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04n_prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04n_prof gpurun_out/r04n_prof k_agg k_dec k_rs k_part k_mm k_group > gpurun_out/r04n_kstats.txt
cat gpurun_out/r04n_kstats.txt

# r04o: one-pass merge with the next range's bounds prefetched, resident persistent grid: parity, timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1
tail -1 gpurun_out/r04o_tests.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/r04o_$i.json 2>&1
  python3 -c "
import json
d = json.loads(open('gpurun_out/r04o_$i.json').read().strip().splitlines()[-1])
print('r04o', $i, {k: d['ms'][k] for k in ('encode_kv', 'dense_to_payload', 'decode', 'decode_sum')})"
done
SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04o_prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04o_prof gpurun_out/r04o_prof k_rs k_dec k_agg k_narrow k_group_prefix k_scan > gpurun_out/r04o_kstats.txt
cat gpurun_out/r04o_kstats.txt

# r04f: dense decode_sum occupancy kernel (parity, A/B, counters); sparse Gradient.sum with narrow
# bins and row-batched MinMax queries (parity, JNI harness, C3 timing A/B), sparse encode PMC
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -m gpu -x -v -k "decode_sum" --timeout 120 --timeout-method thread > gpurun_out/r04f_dsum_tests.log 2>&1
tail -1 gpurun_out/r04f_dsum_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_jni_harness.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py tests/test_gpu_sparse_full.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f_sparse_tests.log 2>&1
tail -1 gpurun_out/r04f_sparse_tests.log
for i in 1 2; do
  SKML_DEC_ROWS_SERIAL=1 SKML_AGG_SEARCH=1 SKML_RS_ROUNDS=1 SKML_DEC_MATERIALIZE=1 timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/r04f_sparse_c3_serial_$i.json 2>&1
  timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/r04f_sparse_c3_$i.json 2>&1
  python3 -c "
import json
for t in ('serial_$i', '$i'):
    d = json.loads(open('gpurun_out/r04f_sparse_c3_%s.json' % t).read().strip().splitlines()[-1])
    print(t, {k: d['ms'][k] for k in ('dense_to_payload', 'encode_kv', 'decode', 'decode_sum')})"
done
bash tools/pmc_decode_sum.sh r04f
bash tools/pmc_sparse.sh r04f

# r04i: two-word flag reads and five-word delta reads in k_dec_lens / k_dec_deltas, wave tiles as the
# aggregate default: parity, end-to-end timing, kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_readobject.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_sparse_tests.log 2>&1
tail -1 gpurun_out/r04i_sparse_tests.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/r04i_new_$i.json 2>&1
  python3 -c "
import json
d = json.loads(open('gpurun_out/r04i_new_$i.json').read().strip().splitlines()[-1])
print('new', $i, d['ms'])"
done
SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i_prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r04i_prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04h_prof_old gpurun_out/r04i_prof k_dec k_agg k_rs k_merge k_narrow k_bin k_group_prefix > gpurun_out/r04i_cmp.txt
cat gpurun_out/r04i_cmp.txt

# r04h: sparse restore / Gradient.sum rework (8,192-key one-pass merge with LDS slots, MODE 1 query,
# key-owner aggregate tiles, two-lane restores): parity, per-kernel A/B against the round-3 forms,
# end-to-end A/B without the profiler, the sparse encode's per-kernel FETCH / WRITE
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04h_sparse_tests.log 2>&1
tail -1 gpurun_out/r04h_sparse_tests.log
LEGACY="SKML_DEC_ROWS_SERIAL=1 SKML_AGG_FORM=s SKML_RS_ROUNDS=1 SKML_AGG_ONE_LANE=1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h_prof_new -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r04h_new_prof.json 2>&1
env $LEGACY timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h_prof_old -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r04h_old_prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04h_prof_old gpurun_out/r04h_prof_new k_ > gpurun_out/r04h_cmp.txt
head -40 gpurun_out/r04h_cmp.txt
for i in 1 2; do
  for V in new:SKML_AB_DEFAULT=1 mode0:SKML_DEC_ROWS_SERIAL=1 rounds:SKML_RS_ROUNDS=1 aggw:SKML_AGG_FORM=w onelane:SKML_AGG_ONE_LANE=1; do
    env "${V#*:}" timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04h_${V%%:*}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04h_${V%%:*}_$i.json').read().strip().splitlines()[-1])
print('${V%%:*}', $i, {k: d['ms'][k] for k in ('encode_kv', 'decode', 'decode_sum')})"
  done
  env $LEGACY timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04h_legacy_$i.json 2>&1
  python3 -c "
import json
d = json.loads(open('gpurun_out/r04h_legacy_$i.json').read().strip().splitlines()[-1])
print('legacy', $i, {k: d['ms'][k] for k in ('encode_kv', 'decode', 'decode_sum')})"
done
bash tools/pmc_sparse.sh r04h

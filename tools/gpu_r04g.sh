# r04g: per-kernel A/B of the sparse decode (default vs the round-3 forms), the decode_sum counters
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_prof_new -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r04g_new.json 2>&1
SKML_DEC_ROWS_SERIAL=1 SKML_AGG_SEARCH=1 SKML_RS_ROUNDS=1 SKML_DEC_MATERIALIZE=1 SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_prof_old -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r04g_old.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04g_prof_old gpurun_out/r04g_prof_new > gpurun_out/r04g_cmp.txt
head -45 gpurun_out/r04g_cmp.txt
bash tools/pmc_decode_sum.sh r04g
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04g_sparse_tests.log 2>&1
tail -1 gpurun_out/r04g_sparse_tests.log

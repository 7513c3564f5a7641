# r05m: Gradient.sum with the sum tile in LDS (parity, A/B against HEAD)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05m
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py > gpurun_out/r05m/tests.log 2>&1
tail -2 gpurun_out/r05m/tests.log
bash tools/ab.sh rmw 2 sparse old=lib:lib_old new= new_pf=form:agg_tiles:4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05m/trace -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r05m/trace.log 2>&1
grep -E "k_agg|k_dec_keys" gpurun_out/r05m/trace/run_kernel_stats.csv | cut -d, -f1-5

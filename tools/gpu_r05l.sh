# r05l: coalesced emission in the pipelined one-pass merge, RsInfo fill and value upload ahead of the decode (parity, A/B against HEAD)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05l
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_readobject.py > gpurun_out/r05l/tests.log 2>&1
tail -2 gpurun_out/r05l/tests.log
bash tools/ab.sh rsemit2 3 restore old=lib:lib_old new=
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05l/trace2 -o run --output-format csv -- python3 tools/bench_sparse.py --reps 5 --only-decode > gpurun_out/r05l/trace2.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05l/trace2 --timeline 18 > gpurun_out/r05l/timeline2.txt
head -20 gpurun_out/r05l/timeline2.txt

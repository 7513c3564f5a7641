# r05k: narrow bins between the values restore's query and the one-pass merge (parity, A/B against r05i)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05k
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_readobject.py > gpurun_out/r05k/tests.log 2>&1
tail -2 gpurun_out/r05k/tests.log
bash tools/ab.sh narrow 3 restore old=lib:lib_old new=
bash tools/ab.sh narrow_s 2 sparse old=lib:lib_old new=
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05k/trace -o run --output-format csv -- python3 tools/bench_sparse.py --reps 5 --only-decode > gpurun_out/r05k/trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05k/trace --timeline 18 > gpurun_out/r05k/timeline.txt
head -20 gpurun_out/r05k/timeline.txt
bash tools/ab.sh xlane 3 dense base= sw16=lib:lib_sw16 sw13=lib:lib_sw13 g8=lib:lib_g8

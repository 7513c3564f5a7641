# r05j: Sort.merge grid sized by occupancy (A/B against r05i's key query build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05j
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py > gpurun_out/r05j/tests.log 2>&1
tail -2 gpurun_out/r05j/tests.log
bash tools/ab.sh rsgrid 3 restore old=lib:lib_old new=
mkdir -p gpurun_out/r05j/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05j/trace -o t -- python tools/bench_sparse.py --reps 5 --only-decode > gpurun_out/r05j/trace.log 2>&1
python tools/trace_gaps.py gpurun_out/r05j/trace --timeline 18 > gpurun_out/r05j/timeline.txt
head -20 gpurun_out/r05j/timeline.txt

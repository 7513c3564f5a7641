# r05f: prefetching Gradient.sum tiles (parity of every form, A/B); the split leaf across sizes;
# the key query's hash / gather ablations on the restore alone; a restore timeline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05f
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py > gpurun_out/r05f/tests.log 2>&1
tail -2 gpurun_out/r05f/tests.log
bash tools/ab.sh pf 3 sparse v1= pf=form:agg_tiles:4
bash tools/ab.sh split26 2 gap26 normal=form:leaf_split:1 split=form:leaf_split:2 h25=form:leaf_split:3
bash tools/ab.sh split24 2 gap24 normal=form:leaf_split:1 split=form:leaf_split:2
bash tools/ab.sh restore 3 restore base= gat=lib:lib_abl hash=lib:lib_abl2 dm1=lib:lib_dm1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r05f/rs_trace -o run --output-format csv -- python3 tools/bench_sparse.py --only-decode --reps 3 > gpurun_out/r05f/rs_trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05f/rs_trace --timeline 16 > gpurun_out/r05f/rs_timeline.txt
head -20 gpurun_out/r05f/rs_timeline.txt
find gpurun_out/r05f -name "*.csv" -size +20M -delete

# r05p: Gradient.sum's run bounds written by the key query (parity, A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05p
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py > gpurun_out/r05p/tests.log 2>&1
tail -2 gpurun_out/r05p/tests.log
bash tools/ab.sh fusedb 3 sparse old=lib:lib_old new= pass=form:agg_bounds:1

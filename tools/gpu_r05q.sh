# r05q: Sort.merge's key-range bounds written by the key query (parity, A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05q
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_readobject.py > gpurun_out/r05q/tests.log 2>&1
tail -2 gpurun_out/r05q/tests.log
bash tools/ab.sh rsfused 3 restore old=lib:lib_old new= pass=form:run_bounds:1

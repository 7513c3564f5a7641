# r05r: narrow table built by extra blocks of the lengths launch (parity, A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05r
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_readobject.py > gpurun_out/r05r/tests.log 2>&1
tail -2 gpurun_out/r05r/tests.log
bash tools/ab.sh narrowfuse 3 restore old=lib:lib_old new=
bash tools/ab.sh narrowfuse_s 2 sparse old=lib:lib_old new=

# r05i: key query with 24-bit BKDR multiplies and the 32-bit modulus (parity, A/B against r05h)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05i
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py > gpurun_out/r05i/tests.log 2>&1
tail -2 gpurun_out/r05i/tests.log
bash tools/ab.sh decm 3 restore old=lib:lib_old new=
bash tools/ab.sh decm_s 2 sparse old=lib:lib_old new=

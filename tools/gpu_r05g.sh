# r05g: the pipelined one-pass Sort.merge (restore) and the new defaults (split leaf, prefetching
# Gradient.sum tiles): parity, then A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05g
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py tests/test_gpu_dense.py > gpurun_out/r05g/tests.log 2>&1
tail -2 gpurun_out/r05g/tests.log
bash tools/ab.sh rsmerge 3 restore pf= plain=form:rs_rounds:2
bash tools/ab.sh sparse5 2 sparse cur=

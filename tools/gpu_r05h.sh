# r05h: persistent key query (parity, A/B) and the restore's counters
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05h
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_full.py > gpurun_out/r05h/tests.log 2>&1
tail -2 gpurun_out/r05h/tests.log
bash tools/ab.sh decp 3 restore pers= tile=form:dec_rows_serial:2
bash tools/pmc_restore.sh r05h

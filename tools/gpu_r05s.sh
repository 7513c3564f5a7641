# r05s: sum-tile presence bits per payload spread over 64 words (parity, A/B, counters)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05s
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py > gpurun_out/r05s/tests.log 2>&1
tail -2 gpurun_out/r05s/tests.log
bash tools/ab.sh hbits 3 sparse old=lib:lib_old new=
bash tools/pmc_agg.sh r05s > /dev/null
python3 -c "
import json;d=json.load(open('gpurun_out/pmc_agg_r05s/summary.json'))['kernels']['k_agg_vtiles_rmw']
print({k: round(v) for k, v in d.items()})"

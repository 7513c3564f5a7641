# r05n: XCD-segmented tile walk, per-wave piece table, two tiles prefetched in the sum-tile kernel (parity, A/B, counters)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05n
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py > gpurun_out/r05n/tests.log 2>&1
tail -2 gpurun_out/r05n/tests.log
bash tools/ab.sh pf2 2 sparse old=lib:lib_old new=
bash tools/pmc_agg.sh r05n2 > /dev/null
python3 -c "
import json;d=json.load(open('gpurun_out/pmc_agg_r05n2/summary.json'))['kernels']['k_agg_vtiles_rmw']
print({k: round(v) for k, v in d.items()})"

# r05c: the changed sparse / dense tests, then the bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05c
set -e
( while sleep 30; do date +%s >> gpurun_out/r05c/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_sparse_exchange.py tests/test_gpu_dense.py tests/test_gpu_sparse.py -k "not test_sparse_shapes" > gpurun_out/r05c/tests.log 2>&1
tail -3 gpurun_out/r05c/tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05c/bench.json 2> gpurun_out/r05c/bench.err
python -c "
import json; d=json.load(open('gpurun_out/r05c/bench.json')); e=d['extras']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], e['ms_per_step_leaf_evented'], e['warmup_steps_run'], e['kernels']); print(json.dumps(e['other_configs']['sparse_aggregate'])[:400])"

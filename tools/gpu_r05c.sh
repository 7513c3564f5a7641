# r05c: the changed sparse / dense tests, then the bench line and the kernel-boundary gaps
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
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r05c/trace -o run --output-format csv -- python3 tools/leaf_gap.py --steps 20 --reps 1 > gpurun_out/r05c/trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05c/trace --skip 200 > gpurun_out/r05c/gaps.json
cat gpurun_out/r05c/gaps.json
find gpurun_out/r05c -name "*.csv" -size +20M -delete
SKML_LIB=sketchml_amd/lib_prof/libskml.so timeout -k 10 120 python tools/prof_leaf_waves.py 268435456 > gpurun_out/r05c/leaf_waves.txt 2>&1
cat gpurun_out/r05c/leaf_waves.txt
bash tools/ab.sh agg 2 sparse v1= v2=form:agg_tiles:3 v4=form:agg_tiles:2 w=form:agg_tiles:1

# r04q: Gradient.sum with one wave per 512-key tile (k_agg_vtiles): parity of every tile form, timing A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_exchange.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1
tail -1 gpurun_out/r04q_tests.log
for i in 1 2 3; do
  for V in vtile:SKML_AB_DEFAULT=1 wave:SKML_AGG_FORM=w; do
    env "${V#*:}" timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04q_${V%%:*}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04q_${V%%:*}_$i.json').read().strip().splitlines()[-1])
print('${V%%:*}', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
done
SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04q_prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04q_prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04q_prof gpurun_out/r04q_prof k_agg k_dec > gpurun_out/r04q_kstats.txt
cat gpurun_out/r04q_kstats.txt

# r04x: wave-per-payload tiles (global loads) with presence bits per (payload, key) as the default;
# vtile = SKML_AGG_FORM=v.  Parity (incl. keys repeated across groups), timing, kernel stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04x
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04x/tests.log 2>&1
tail -1 gpurun_out/r04x/tests.log
for i in 1 2 3; do
  for V in "wave:SKML_AB_DEFAULT=1" "vtile:SKML_AGG_FORM=v"; do
    N=${V%%:*}
    env ${V#*:} timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04x/${N}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04x/${N}_$i.json').read().strip().splitlines()[-1])
print('$N', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
done
SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04x/prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04x/prof.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04x/prof gpurun_out/r04x/prof k_agg k_dec k_rs > gpurun_out/r04x/kstats.txt
cat gpurun_out/r04x/kstats.txt

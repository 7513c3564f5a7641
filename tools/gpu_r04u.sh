# r04u: XCD-aware tile walk (each XCD's units take consecutive tiles per round) vs the plain
# strided walk, for the staged wave tiles and the wave-per-payload tiles.  Parity, timing, stats.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04u
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04u/tests.log 2>&1
tail -1 gpurun_out/r04u/tests.log
for i in 1 2 3; do
  for V in "vtile:SKML_AB_DEFAULT=1" "vtile_plain:SKML_AGG_WALK=plain" "wave:SKML_AGG_FORM=w" "wave_plain:SKML_AGG_FORM=w SKML_AGG_WALK=plain"; do
    N=${V%%:*}
    env ${V#*:} timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04u/${N}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04u/${N}_$i.json').read().strip().splitlines()[-1])
print('$N', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
done
for V in "vtile:SKML_AB_DEFAULT=1" "vtile_plain:SKML_AGG_WALK=plain"; do
  N=${V%%:*}
  env ${V#*:} SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u/prof_$N -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04u/prof_$N.json 2>&1
done
python3 tools/kstats_cmp.py gpurun_out/r04u/prof_vtile gpurun_out/r04u/prof_vtile_plain k_agg k_dec k_rs > gpurun_out/r04u/kstats.txt
cat gpurun_out/r04u/kstats.txt

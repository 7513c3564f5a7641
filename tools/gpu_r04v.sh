# r04v: payload-pointer loads as global (address space 1) loads instead of flat loads (which also
# count on lgkmcnt, so every LDS wait waited for them): Gradient.sum tiles, and k_decode_sum_occ's
# codes.  prev = the previous commit's library (sketchml_amd/lib_prev), new = this tree's.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04v
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse.py tests/test_gpu_dense.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04v/tests.log 2>&1
tail -1 gpurun_out/r04v/tests.log
for i in 1 2 3; do
  for V in "prev:SKML_LIB=sketchml_amd/lib_prev/libskml.so" "new:SKML_AB_DEFAULT=1" "new_wave:SKML_AGG_FORM=w"; do
    N=${V%%:*}
    env ${V#*:} timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04v/${N}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04v/${N}_$i.json').read().strip().splitlines()[-1])
print('$N', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
  for V in "prev:SKML_LIB=sketchml_amd/lib_prev/libskml.so" "new:SKML_AB_DEFAULT=1"; do
    N=${V%%:*}
    env ${V#*:} timeout -k 10 120 python tools/bench_decode_sum.py --bins 129 > gpurun_out/r04v/dsum_${N}_$i.json 2>&1
    echo "dsum $N $i $(tail -1 gpurun_out/r04v/dsum_${N}_$i.json)"
  done
done
for V in "new:SKML_AB_DEFAULT=1" "new_wave:SKML_AGG_FORM=w"; do
  N=${V%%:*}
  env ${V#*:} SKML_AGG_ONE_LANE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04v/prof_$N -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r04v/prof_$N.json 2>&1
done
python3 tools/kstats_cmp.py gpurun_out/r04v/prof_new gpurun_out/r04v/prof_new_wave k_agg k_dec k_rs > gpurun_out/r04v/kstats.txt
cat gpurun_out/r04v/kstats.txt

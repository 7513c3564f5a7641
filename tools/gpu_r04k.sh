# r04k: MinMax scatter hashing the keys again (no cell array) and the run-ranked partition scatter,
# each against its previous form: parity and the C3 encode A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_full.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k_sparse_tests.log 2>&1
tail -1 gpurun_out/r04k_sparse_tests.log
for i in 1 2 3; do
  for V in new:SKML_AB_DEFAULT=1 cells:SKML_MM_CELLS=1 ballot:SKML_PART_BALLOT=1; do
    env "${V#*:}" timeout -k 10 200 python tools/bench_sparse.py --reps 10 --only-e2e > gpurun_out/r04k_${V%%:*}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04k_${V%%:*}_$i.json').read().strip().splitlines()[-1])
print('${V%%:*}', $i, d)"
  done
done
SKML_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_prof -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --only-e2e > gpurun_out/r04k_prof.json 2>&1
SKML_SERIAL=1 SKML_MM_CELLS=1 SKML_PART_BALLOT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04k_prof_old -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --only-e2e > gpurun_out/r04k_prof_old.json 2>&1
python3 tools/kstats_cmp.py gpurun_out/r04k_prof_old gpurun_out/r04k_prof k_ > gpurun_out/r04k_cmp.txt
head -25 gpurun_out/r04k_cmp.txt

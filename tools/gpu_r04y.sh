# r04y: Gradient.sum with the payload restores on two streams (default) vs one (SKML_AGG_ONE_LANE=1), ms
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04y
set -e
for i in 1 2 3; do
  for V in "two:SKML_AB_DEFAULT=1" "one:SKML_AGG_ONE_LANE=1"; do
    N=${V%%:*}
    env ${V#*:} timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04y/${N}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04y/${N}_$i.json').read().strip().splitlines()[-1])
print('$N', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
done

#!/bin/bash
# Round evidence set (GPU box): the GPU suite, smoke(), the default bench line (the 2^28 north
# star), the rocprof profile set of tools/prof_round.sh and the C3 sparse bench.
# usage (through gpurun): bash tools/final_evidence.sh TAG [skip-tests | tests-only]
TAG=${1:-cur}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# a heartbeat under gpurun_out/ while long, quiet steps (the oracle's 2^30 sketch) run
( while sleep 30; do date +%s >> gpurun_out/${TAG}_heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
  tail -1 gpurun_out/${TAG}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  tail -1 gpurun_out/${TAG}_smoke.log
fi
[ "$2" = "tests-only" ] && exit 0
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tail -c 400 gpurun_out/${TAG}_bench.json
bash tools/prof_round.sh "$TAG"
timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/${TAG}_sparse_c3_bench.json 2>&1
tail -c 600 gpurun_out/${TAG}_sparse_c3_bench.json
bash tools/pmc_sparse.sh "$TAG" > /dev/null

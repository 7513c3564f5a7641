#!/bin/bash
# Round-end evidence set (GPU box): the GPU suite, smoke(), the default bench line, the rocprof
# profile set of tools/prof_round.sh and the C3 sparse bench.  usage (through gpurun): bash tools/final_evidence.sh TAG
TAG=${1:-cur}
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tail -c 400 gpurun_out/${TAG}_bench.json
bash tools/prof_round.sh "$TAG"
timeout -k 10 200 python tools/bench_sparse.py --reps 10 --aggregate 8 > gpurun_out/${TAG}_sparse_c3_bench.json 2>&1
tail -c 600 gpurun_out/${TAG}_sparse_c3_bench.json

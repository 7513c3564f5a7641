# rocprofv3 kernel trace of the C3 sparse bench (GPU box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sp -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 > gpurun_out/prof_sp.json

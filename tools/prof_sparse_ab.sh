# rocprofv3 kernel stats of the C3 sparse bench for several in-tree builds (GPU box)
#   bash tools/prof_sparse_ab.sh lib lib_c0 lib_c1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in "$@"; do
  SKML_LIB=sketchml_amd/$L/libskml.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$L -o run \
    --output-format csv -- python3 tools/bench_sparse.py --reps 3 > gpurun_out/ab_$L.json
done

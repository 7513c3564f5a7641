#!/bin/bash
# rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs) over one C3 sparse encode (GPU box), folded
# per kernel by tools/pmc_sparse_summary.py into gpurun_out/pmc_sp_TAG/sparse_pmc.json: HBM bytes per
# launch of every kernel of dense -> payload, their sum and its ratio to the 6.2 B/element
# algorithmic bytes of SURVEY §8(d).  usage (through gpurun): bash tools/pmc_sparse.sh TAG
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_sp_$TAG
mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --only-e2e > $OUT/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --only-e2e > $OUT/write.log 2>&1
python3 tools/pmc_sparse_summary.py --fetch $OUT/fetch --write $OUT/write --out $OUT/sparse_pmc.json
find "$OUT" -name "*counter_collection.csv" -size +20M -delete
find "$OUT" -name "*kernel_trace.csv" -size +20M -delete

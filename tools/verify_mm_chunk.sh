#!/bin/bash
# GPU check of tools/patches/mm_chunk_runtime.diff built as sketchml_amd/lib_mmc (make OUT=../lib_mmc after git apply):
# the sparse GPU suites on that build, then an A/B against the default lib.  usage (through gpurun): bash tools/verify_mm_chunk.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SKML_LIB=sketchml_amd/lib_mmc/libskml.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_sparse_full.py tests/test_gpu_sparse_exchange.py tests/test_gpu_sparse_readobject.py > gpurun_out/t_mmc.log 2>&1
tail -1 gpurun_out/t_mmc.log
LIBS="lib lib_mmc" REPS=4 bash tools/ab_sparse_libs.sh 2>&1 | tee gpurun_out/ab_mmc.txt

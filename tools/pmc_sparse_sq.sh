# one SQ counter pass over the C3 sparse bench (GPU box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_sp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-include-regex 'k_(compact|part|group_prep|mm_|delta)' -d gpurun_out/pmc_sp/sq -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 > /dev/null
python3 tools/pmc_kernels.py gpurun_out/pmc_sp/sq.json gpurun_out/pmc_sp/sq/run_counter_collection.csv

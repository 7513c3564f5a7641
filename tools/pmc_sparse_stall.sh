# one SQ stall-breakdown counter pass over the C3 sparse bench (GPU box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_sp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex 'k_(compact|part|group_prep|mm_|delta)' -d gpurun_out/pmc_sp/stall -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 > /dev/null
python3 tools/pmc_kernels.py gpurun_out/pmc_sp/stall.json gpurun_out/pmc_sp/stall/run_counter_collection.csv

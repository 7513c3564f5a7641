# SQ stall / instruction and L2 hit counter passes over the sparse restore and Gradient.sum
# kernels (tools/bench_sparse.py --aggregate 2; GPU box).  One --pmc pass per run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_dec
RX='k_(dec_|agg_|narrow)'
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex "$RX" -d gpurun_out/pmc_dec/sq -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --aggregate 2 > /dev/null
python3 tools/pmc_kernels.py gpurun_out/pmc_dec/sq.json gpurun_out/pmc_dec/sq/run_counter_collection.csv
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" -d gpurun_out/pmc_dec/tcc -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --aggregate 2 > /dev/null
python3 tools/pmc_kernels.py gpurun_out/pmc_dec/tcc.json gpurun_out/pmc_dec/tcc/run_counter_collection.csv
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d gpurun_out/pmc_dec/fetch -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --aggregate 2 > /dev/null
python3 tools/pmc_kernels.py gpurun_out/pmc_dec/fetch.json gpurun_out/pmc_dec/fetch/run_counter_collection.csv

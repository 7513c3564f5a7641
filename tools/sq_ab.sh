# SQ counters of bench.py's kernels for the default lib and sketchml_amd/lib_v1 (A/B, GPU box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sq_ab
for L in ${LIBS:-lib lib_v1}; do
  SKML_LIB=sketchml_amd/$L/libskml.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    -d gpurun_out/sq_ab/$L -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > gpurun_out/sq_ab/$L.log 2>&1
  python3 tools/pmc_kernels.py gpurun_out/sq_ab/$L.json gpurun_out/sq_ab/$L/run_counter_collection.csv
done

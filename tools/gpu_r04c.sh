cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 60 tools/ubench/min3_probe > gpurun_out/r04c_min3_probe.txt 2>&1 || true
cat gpurun_out/r04c_min3_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -m gpu -x -v -k "decode_sum" --timeout 120 --timeout-method thread > gpurun_out/r04c_dsum_tests.log 2>&1
tail -2 gpurun_out/r04c_dsum_tests.log
bash tools/pmc_decode_sum.sh r04c
bash tools/ab_libs.sh 2 268435456 2 lib lib_swz lib_swz8 2>&1 | tee gpurun_out/r04c_ab_leaf.txt
SKML_LIB=sketchml_amd/lib_swz/libskml.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_swz_dense_tests.log 2>&1
tail -2 gpurun_out/r04c_swz_dense_tests.log

# r04e: decode_sum occupancy kernel: parity (all variants) + A/B + counters
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -m gpu -x -v -k "decode_sum" --timeout 120 --timeout-method thread > gpurun_out/r04e_dsum_tests.log 2>&1
tail -1 gpurun_out/r04e_dsum_tests.log
bash tools/pmc_decode_sum.sh r04e

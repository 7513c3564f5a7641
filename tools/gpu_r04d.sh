# r04d: decode_sum (rep vs software-pipelined plain), leaf A/B (base vs sort4+min3det vs +swizzle),
# dense parity of the new leaf.  usage (through gpurun): bash tools/gpu_r04d.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py -m gpu -x -v -k "decode_sum" --timeout 120 --timeout-method thread > gpurun_out/r04d_dsum_tests.log 2>&1
tail -1 gpurun_out/r04d_dsum_tests.log
for i in 1 2 3; do
  SKML_DECODE_SUM_PLAIN=1 timeout -k 10 120 python3 tools/bench_decode_sum.py >> gpurun_out/r04d_dsum_plainpf.jsonl
  timeout -k 10 120 python3 tools/bench_decode_sum.py >> gpurun_out/r04d_dsum_rep.jsonl
done
tail -n 3 gpurun_out/r04d_dsum_plainpf.jsonl gpurun_out/r04d_dsum_rep.jsonl
bash tools/ab_libs.sh 2 268435456 2 lib_base lib lib_s4swz 2>&1 | tee gpurun_out/r04d_ab_leaf.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_golden.py tests/test_gpu_configs.py -m gpu -x -q -k "not c5_whole and not c4_eight" --timeout 300 --timeout-method thread > gpurun_out/r04d_dense_tests.log 2>&1
tail -1 gpurun_out/r04d_dense_tests.log

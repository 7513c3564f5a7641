# C5 shapes: 2^27 floats per GPU with 4 bins (2-bit codes), and the whole 2^30-float gradient on one GPU
set -e
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline --n 134217728 --bins 4 --buffers 2 > gpurun_out/b_c5_shard.json
timeout -k 10 300 python bench.py --no-cpu-baseline --n 1073741824 --bins 4 --buffers 1 --steps 5 --warmup 2 > gpurun_out/b_c5_full.json

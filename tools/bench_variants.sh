set -e
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_f32.json
timeout -k 10 200 python bench.py --no-cpu-baseline --dtype f64 --steps 10 > gpurun_out/b_f64.json
timeout -k 10 200 python bench.py --no-cpu-baseline --quant uniform > gpurun_out/b_u32.json
timeout -k 10 200 python bench.py --no-cpu-baseline --quant uniform --dtype f64 > gpurun_out/b_u64.json

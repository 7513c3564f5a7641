# rocprofv3 kernel stats of the bench variants (fp64 quantile, uniform fp32/fp64)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "--dtype f64" "--quant uniform" "--quant uniform --dtype f64"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 10 $v > gpurun_out/prof_$tag.json
done

#!/bin/bash
# rocprofv3 kernel stats of the non-default dense shapes the bench line reports under
# extras.other_configs (GPU box): the north-star 2^28-float encode, the fp64 bucket and the
# uniform quantizer.  usage (through gpurun): bash tools/prof_configs.sh TAG
#   -> gpurun_out/profc_TAG/{n2p28,f64,uniform}/ (stats csv + the bench line of that run)
set -e
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/profc_$TAG
mkdir -p "$OUT"
run() {  # name, bench args...
    local name=$1
    shift
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline --no-configs --no-extras "$@" > "$OUT/$name.json" 2> "$OUT/$name.log"
    find "$OUT/$name" -name "*kernel_trace.csv" -size +20M -delete
}
run n2p28 --n 268435456 --steps 20 --warmup 5 --buffers 1
run f64 --dtype f64 --steps 20 --warmup 5
run uniform --quant uniform --steps 20 --warmup 5
run uniform_f64 --quant uniform --dtype f64 --steps 20 --warmup 5

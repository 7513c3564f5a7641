cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05a && timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err && python -c "
import json; d=json.load(open('gpurun_out/r05a/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['extras']['kernels'])"

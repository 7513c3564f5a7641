# r05b: the headline's time outside the kernels (tools/leaf_gap.py) + a kernel-trace timeline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05b
set -e
timeout -k 10 200 python tools/leaf_gap.py --steps 20 --reps 3 > gpurun_out/r05b/leaf_gap.jsonl 2>&1
tail -1 gpurun_out/r05b/leaf_gap.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r05b/trace -o run --output-format csv -- python3 tools/leaf_gap.py --steps 20 --reps 1 > gpurun_out/r05b/trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05b/trace > gpurun_out/r05b/gaps.json
cat gpurun_out/r05b/gaps.json
find gpurun_out/r05b -name "*.csv" -size +20M -delete

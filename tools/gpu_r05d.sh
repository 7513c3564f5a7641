# r05d: kernel-boundary gaps, the leaf's per-wave profile, Gradient.sum tile A/B, the gather ablation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05d
set -e
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r05d/trace -o run --output-format csv -- python3 tools/leaf_gap.py --steps 20 --reps 1 > gpurun_out/r05d/trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05d/trace --skip 200 > gpurun_out/r05d/gaps.json
cat gpurun_out/r05d/gaps.json
find gpurun_out/r05d -name "*.csv" -size +20M -delete
SKML_LIB=sketchml_amd/lib_prof/libskml.so timeout -k 10 120 python tools/prof_leaf_waves.py 268435456 > gpurun_out/r05d/leaf_waves.txt 2>&1
cat gpurun_out/r05d/leaf_waves.txt
bash tools/ab.sh agg 2 sparse v1= v2=form:agg_tiles:3 v4=form:agg_tiles:2 w=form:agg_tiles:1
bash tools/ab.sh gather 2 sparse base= abl=lib:lib_abl
SKML_LIB=sketchml_amd/lib_profs/libskml.so timeout -k 10 120 python tools/prof_merge.py 268435456 > gpurun_out/r05d/merge_phases.txt 2>&1
tail -3 gpurun_out/r05d/merge_phases.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05d/sparse_stats -o run --output-format csv -- python3 tools/bench_sparse.py --reps 3 --aggregate 8 > gpurun_out/r05d/sparse_stats.log 2>&1
python3 tools/kstats_cmp.py gpurun_out/r05d/sparse_stats gpurun_out/r05d/sparse_stats > gpurun_out/r05d/sparse_kernel_stats.txt 2>&1 || true
head -40 gpurun_out/r05d/sparse_kernel_stats.txt
find gpurun_out/r05d -name "*kernel_trace.csv" -size +20M -delete
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r05d/sp_trace -o run --output-format csv -- python3 tools/bench_sparse.py --only-e2e --reps 3 > gpurun_out/r05d/sp_trace.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r05d/sp_trace --timeline 45 > gpurun_out/r05d/sp_timeline.txt
head -50 gpurun_out/r05d/sp_timeline.txt
find gpurun_out/r05d -name "*.csv" -size +20M -delete
bash tools/ab.sh qstore 3 dense q0= q1=lib:lib_q1 q2=lib:lib_q2

# r05t: ablations of the sum-tile kernel (the adds into the tile; the sum's stores), kernel times under rocprof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05t
set -e
for V in base: rmw:sketchml_amd/lib_abl_rmw/libskml.so st:sketchml_amd/lib_abl_st/libskml.so; do
  NAME=${V%%:*}; LIB=${V#*:}
  if [ -n "$LIB" ]; then export SKML_LIB=$LIB; else unset SKML_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05t/$NAME -o run --output-format csv -- python3 tools/bench_sparse.py --reps 2 --aggregate 8 > gpurun_out/r05t/$NAME.log 2>&1
  python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('gpurun_out/r05t/$NAME/**/run_kernel_stats.csv', recursive=True)[0])):
    if 'k_agg' in r['Name'] or 'k_dec_keys' in r['Name']: print('$NAME', r['Name'].split('(')[0][-32:], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done

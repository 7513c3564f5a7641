# r05e: the leaf's tail: one-wave-per-tile against the split leaf (four waves per tile) at 2^28
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05e
set -e
bash tools/ab.sh split 2 gap normal=form:leaf_split:1 split=form:leaf_split:2
SKML_TOOL_FORMS=leaf_split:1 SKML_LIB=sketchml_amd/lib_prof/libskml.so timeout -k 10 120 python tools/prof_leaf_waves.py 268435456 > gpurun_out/r05e/leaf_waves.txt 2>&1
cat gpurun_out/r05e/leaf_waves.txt
bash tools/ab.sh hybrid 3 gap normal=form:leaf_split:1 h25= h12=form:leaf_split:4 h50=form:leaf_split:5
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dense.py -k "leaf_forms or large or quantize_matches" > gpurun_out/r05e/tests.log 2>&1
tail -3 gpurun_out/r05e/tests.log
bash tools/ab.sh decq 2 sparse base= dm1=lib:lib_dm1 gat=lib:lib_abl hash=lib:lib_abl2
SKML_LIB=sketchml_amd/lib_dm1/libskml.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_sparse_full.py -k "restore or shapes or c3_full or edge or f64" > gpurun_out/r05e/dm1_tests.log 2>&1
tail -2 gpurun_out/r05e/dm1_tests.log

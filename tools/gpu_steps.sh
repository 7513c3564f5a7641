#!/bin/bash
# One GPU session of named steps, in order (through gpurun).  Every step writes under
# gpurun_out/TAG/ (or where the script it calls writes) and runs under its own time limit; the
# session stops at the first failing step.  tools/RUNS.md lists the round's sessions as calls of
# this script.
#
#   bash tools/gpu_steps.sh TAG STEP [STEP ...]
#
# STEP:
#   tests:FILE[+FILE...][@K]  pytest -m gpu on tests/FILE.py ... (-k K if given) -> TAG/tests.log
#   suite                     the whole GPU suite and smoke() (tools/final_evidence.sh TAG tests-only)
#   abtests                   the tests of the A/B-only kernel forms against sketchml_amd/lib_ab (make -C sketchml_amd/csrc ab)
#   bench                     python bench.py --gpus 1 --steps 20 --warmup 5 -> TAG/bench.json
#   ab:NAME:REPS:KIND:VARIANT[+VARIANT...]   tools/ab.sh NAME REPS KIND VARIANT ... (see ab.sh)
#   pmc:agg | pmc:restore | pmc:sparse       the counter passes (tools/pmc_*.sh TAG)
#   timeline:KIND[:N]         rocprofv3 --kernel-trace --memory-copy-trace over tools/bench_sparse.py
#                             (KIND: restore = --only-decode, encode = --only-e2e, aggregate =
#                             --aggregate 8), the last N operations -> TAG/KIND_timeline.txt
#   kstats:KIND[:LIB]         rocprofv3 --kernel-trace --stats over the same (with sketchml_amd/LIB/libskml.so
#                             if given) -> TAG/KIND[_LIB]_kernel_stats.csv
#   hiptrace[:KIND]           HIP API + kernel trace of the C3 encode (or KIND as in timeline) -> TAG/hiptrace/
#   leafgap                   tools/leaf_gap.py (clean / evented / synchronised encode blocks)
#   leafwaves[:LIB]           tools/prof_leaf_waves.py at 2^28 (a SKML_PROF_LEAF build in LIB)
#   mergephases[:LIB]         tools/prof_merge.py at 2^28 (a SKML_PROF_SUMMARY build in LIB)
#   batchtrace[:ARGS]         rocprofv3 --kernel-trace over tools/batch_probe.py ARGS -> TAG/batch_timeline.txt
#   ubench:NAME               tools/ubench/bin/NAME (built here: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/bin/NAME tools/ubench/NAME.hip)
# Per-variant libraries and kernel forms go through ab.sh's variants (lib:DIR, form:NAME:VALUE).
set -e
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
sparse_args() {
  case $1 in
    restore) echo "--only-decode --reps 5" ;;
    encode) echo "--only-e2e --reps 3" ;;
    aggregate) echo "--aggregate 8 --reps 3" ;;
    *) echo "unknown kind $1" >&2; return 2 ;;
  esac
}
for STEP in "$@"; do
  echo "== $STEP"
  case $STEP in
    tests:*)
      SPEC=${STEP#tests:}
      K=""
      if [[ $SPEC == *@* ]]; then K=${SPEC#*@}; SPEC=${SPEC%%@*}; fi
      FILES=$(echo "$SPEC" | tr '+' '\n' | sed 's|^|tests/|; s|$|.py|' | tr '\n' ' ')
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $FILES ${K:+-k "$K"} \
        > "$OUT/tests.log" 2>&1
      tail -2 "$OUT/tests.log" ;;
    suite)
      bash tools/final_evidence.sh "$TAG" tests-only ;;
    abtests)
      SKML_LIB=sketchml_amd/lib_ab/libskml.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 \
        --timeout-method thread -m "gpu and ab" > "$OUT/ab_tests.log" 2>&1
      tail -2 "$OUT/ab_tests.log" ;;
    bench)
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
      tail -c 300 "$OUT/bench.json" ;;
    ab:*)
      IFS=':' read -r _ NAME REPS KIND VARS <<< "$STEP"
      bash tools/ab.sh "$NAME" "$REPS" "$KIND" $(echo "$VARS" | tr '+' ' ') ;;
    pmc:agg) bash tools/pmc_agg.sh "$TAG" > /dev/null ;;
    pmc:restore) bash tools/pmc_restore.sh "$TAG" > /dev/null ;;
    pmc:sparse) bash tools/pmc_sparse.sh "$TAG" > /dev/null ;;
    timeline:*)
      IFS=':' read -r _ KIND N <<< "$STEP"
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/${KIND}_trace" -o run --output-format csv \
        -- python3 tools/bench_sparse.py $(sparse_args "$KIND") > "$OUT/${KIND}_trace.log" 2>&1
      python3 tools/trace_gaps.py "$OUT/${KIND}_trace" --timeline "${N:-20}" > "$OUT/${KIND}_timeline.txt"
      head -"${N:-20}" "$OUT/${KIND}_timeline.txt"
      find "$OUT" -name "*.csv" -size +20M -delete ;;
    kstats:*)
      IFS=':' read -r _ KIND LIB <<< "$STEP"
      NAME=${KIND}${LIB:+_$LIB}
      (
        if [ -n "$LIB" ]; then export SKML_LIB=sketchml_amd/$LIB/libskml.so; fi
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${NAME}_stats" -o run --output-format csv \
          -- python3 tools/bench_sparse.py $(sparse_args "$KIND") > "$OUT/${NAME}_stats.log" 2>&1
      )
      cp "$(find "$OUT/${NAME}_stats" -name '*kernel_stats.csv' | head -1)" "$OUT/${NAME}_kernel_stats.csv"
      find "$OUT" -name "*kernel_trace.csv" -size +20M -delete ;;
    hiptrace*)
      KIND=${STEP#hiptrace}; KIND=${KIND#:}
      if [ -n "$KIND" ]; then ARGS=$(sparse_args "$KIND"); else ARGS="--reps 3 --only-e2e"; fi
      timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d "$OUT/hiptrace" -o run \
        --output-format csv -- python3 tools/bench_sparse.py $ARGS > "$OUT/hiptrace.log" 2>&1
      find "$OUT" -name "*.csv" -size +30M -delete ;;
    leafgap)
      timeout -k 10 200 python tools/leaf_gap.py --steps 20 --reps 3 > "$OUT/leaf_gap.jsonl" 2>&1
      tail -1 "$OUT/leaf_gap.jsonl" ;;
    leafwaves*)
      LIB=${STEP#leafwaves}; LIB=${LIB#:}
      SKML_LIB=sketchml_amd/${LIB:-lib_prof}/libskml.so timeout -k 10 120 python tools/prof_leaf_waves.py 268435456 \
        > "$OUT/leaf_waves.txt" 2>&1
      tail -5 "$OUT/leaf_waves.txt" ;;
    mergephases*)
      LIB=${STEP#mergephases}; LIB=${LIB#:}
      SKML_LIB=sketchml_amd/${LIB:-lib_profs}/libskml.so timeout -k 10 120 python tools/prof_merge.py 268435456 \
        > "$OUT/merge_phases.txt" 2>&1
      tail -3 "$OUT/merge_phases.txt" ;;
    batchtrace*)
      ARGS=${STEP#batchtrace}; ARGS=${ARGS#:}
      timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/batch_trace" -o run --output-format csv \
        -- python3 tools/batch_probe.py $ARGS > "$OUT/batch_trace.log" 2>&1
      python3 tools/trace_gaps.py "$OUT/batch_trace" --timeline 60 > "$OUT/batch_timeline.txt"
      tail -1 "$OUT/batch_trace.log"
      find "$OUT" -name "*.csv" -size +20M -delete ;;
    ubench:*)
      NAME=${STEP#ubench:}
      timeout -k 10 300 tools/ubench/bin/"$NAME" > "$OUT/ubench_$NAME.txt" 2>&1
      tail -4 "$OUT/ubench_$NAME.txt" ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
